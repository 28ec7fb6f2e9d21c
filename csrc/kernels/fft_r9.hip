// Transform kernels for the lengths 9*2^k, 144..1152 (radix-9 = 3x3 pass, or 6 x 3).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R9_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

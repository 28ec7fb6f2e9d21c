// Transform kernels for the lengths 15*2^k, 240..1920 (radix-15 = 5x3 pass, or 10 x 3).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R15_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

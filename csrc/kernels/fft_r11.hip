// Transform kernels for the lengths 11*2^k, 176..1408 (radix-11 last pass).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R11_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

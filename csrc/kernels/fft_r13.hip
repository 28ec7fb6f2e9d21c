// Transform kernels for the lengths 13*2^k, 208..1664 (radix-13 last pass).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R13_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

// Transform kernels for the lengths 5*2^k, 80..1280 (radix-5 last pass).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R5_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

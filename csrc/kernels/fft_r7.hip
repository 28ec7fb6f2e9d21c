// Transform kernels for the lengths 7*2^k, 112..1792 (radix-7 last pass).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R7_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

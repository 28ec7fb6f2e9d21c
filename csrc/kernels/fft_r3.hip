// Transform kernels for the lengths 3*2^k, 48..1536 (radix-3 last pass).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_R3_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

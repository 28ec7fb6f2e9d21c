// Transform kernels for length 2048 (fft_pow2.hip holds the shorter powers of two).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_INSTANTIATE(2048)

}  // namespace channel

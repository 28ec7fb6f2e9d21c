// Transform kernels for length 1024 (fft_pow2.hip holds the shorter powers of two).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_INSTANTIATE(1024)

}  // namespace channel

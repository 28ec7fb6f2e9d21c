// Transform kernels for the lengths powers of two, 16..2048.
#include "fft_impl.hpp"

namespace channel {

CH_FFT_POW2_LENGTHS(CH_FFT_INSTANTIATE)

}  // namespace channel

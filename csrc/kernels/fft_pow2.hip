// Transform kernels for the power-of-two lengths 16..512 (1024 and 2048, the heaviest instantiation
// sets, have their own units: fft_pow2_1024.hip, fft_pow2_2048.hip; parallel compilation).
#include "fft_impl.hpp"

namespace channel {

CH_FFT_INSTANTIATE(16)
CH_FFT_INSTANTIATE(32)
CH_FFT_INSTANTIATE(64)
CH_FFT_INSTANTIATE(128)
CH_FFT_INSTANTIATE(256)
CH_FFT_INSTANTIATE(512)

}  // namespace channel

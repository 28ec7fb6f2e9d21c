// K-SPEC reference-parity variant PAR = 1: explicit_d2 = "dd" (D1 o D1 explicit viscous term).
#include "kspec_impl.hpp"

namespace channel {

template void kspec_launch_par<1>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);

}  // namespace channel

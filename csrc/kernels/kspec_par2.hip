// K-SPEC reference-parity variant PAR = 2: influence = "analytic" (cosh/sinh influence functions).
#include "kspec_impl.hpp"

namespace channel {

template void kspec_launch_par<2>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);

}  // namespace channel

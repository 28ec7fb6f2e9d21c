// K-SPEC reference-parity variant PAR = 3: both reference-parity switches.
#include "kspec_impl.hpp"

namespace channel {

template void kspec_launch_par<3>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);

}  // namespace channel

// K-SPEC launcher and its default instantiations (compact D2, discrete Green's functions); the
// kernel is in kspec_impl.hpp, the reference-parity variants in kspec_par*.hip.
#include "kspec_impl.hpp"

namespace channel {

template void kspec_launch_par<0>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);

void kspec_launch(const YTablesDev& t, const SpecArgs& a, bool fp64, hipStream_t stream) {
  CH_CHECK(a.N == t.tab.N, "kspec: NY mismatch with tables");
  CH_CHECK(!a.analytic_influence || a.ygrid, "kspec: analytic influence needs the y grid");
  CH_CHECK(a.lines > 0, "kspec: no lines");
  CH_CHECK(!a.kzb || (a.kzb == kSpecKzBlock && a.nkz % kSpecKzBlock == 0 && a.lines % kSpecKzBlock == 0),
           "kspec: the blocked spectral layout needs whole 8-line kz blocks");
  CH_CHECK(static_cast<long long>(a.N) * a.lines < (1LL << 32), "kspec: field exceeds 32-bit element offsets");
  const int par = (a.explicit_dd ? kParDD : 0) | (a.analytic_influence ? kParAnalytic : 0);
  switch (par) {
    case 0: kspec_launch_par<0>(t, a, fp64, stream); break;
    case kParDD: kspec_launch_par<kParDD>(t, a, fp64, stream); break;
    case kParAnalytic: kspec_launch_par<kParAnalytic>(t, a, fp64, stream); break;
    default: kspec_launch_par<kParDD | kParAnalytic>(t, a, fp64, stream); break;
  }
  HIP_LAUNCH_CHECK(stream);
}

}  // namespace channel

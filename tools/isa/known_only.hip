// dev helper: the f64 PlusTimes rows-known heavy kernel alone, for fast ISA inspection
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I combblas_amd/csrc --cuda-device-only -S tools/isa/known_only.hip
#include "spgemm_kernels.hpp"
namespace cbg {
void launch_known_only(const KnownUnit* ku, const unsigned long long* n, DevCsc<double> A, DevCsc<double> B, Split spl,
                       NumOut<double> o) {
  k_num_heavy_known<Semiring<0, double>, double, CBG_KNOWN_LOGT, CBG_KNOWN_NT, true><<<1, CBG_KNOWN_NT>>>(ku, n, A, B, spl, o, (unsigned long long*)n);
}
}  // namespace cbg

// dev helper: the wide-column symbolic part kernel alone, for fast ISA / resource inspection
#include "spgemm_kernels.hpp"
namespace cbg {
void launch_sym_only(const PartItem* it, const int* n, const int64_t* Acp, const int32_t* Air, const int64_t* Bcp,
                     const int32_t* Bir, const int2* span, Split spl, int64_t* nnz, HeavyOut ho) {
  k_sym_part<kPartNT, true, int32_t><<<1, kPartNT>>>(it, n, 1 << 20, Acp, Air, Bcp, Bir, span, spl, nnz, ho);
}
}  // namespace cbg

// Depth-5 instantiation of the PERFECT-layout tree kernels (see tree_common.h).
#include "tree_common.h"

namespace pmml_tree {
int launch_perfect_d5(hipStream_t st, const TreeArgs& a, dim3 grid, size_t lds) {
  return launch_perfect<5>(st, a, grid, lds);
}
int launch_grouped_d5(hipStream_t st, const TreeArgs& a, const GroupedTreeArgs& g, int tiles, size_t lds) {
  size_t need = 0;
  const int chk = wide_check<5>(a, need);
  return chk ? chk : launch_grouped<5>(st, a, g, tiles, lds);
}
}  // namespace pmml_tree

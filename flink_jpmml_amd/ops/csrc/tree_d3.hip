// Depth-3 instantiation of the PERFECT-layout tree kernels (see tree_common.h).
#include "tree_common.h"

namespace pmml_tree {
int launch_perfect_d3(hipStream_t st, const TreeArgs& a, dim3 grid, size_t lds) {
  return launch_perfect<3>(st, a, grid, lds);
}
int launch_grouped_d3(hipStream_t st, const TreeArgs& a, const GroupedTreeArgs& g, int tiles, size_t lds) {
  size_t need = 0;
  const int chk = wide_check<3>(a, need);
  return chk ? chk : launch_grouped<3>(st, a, g, tiles, lds);
}
}  // namespace pmml_tree

// Depth-1 instantiation of the PERFECT-layout tree kernels (see tree_common.h).
#include "tree_common.h"

namespace pmml_tree {
int launch_perfect_d1(hipStream_t st, const TreeArgs& a, dim3 grid, size_t lds) {
  return launch_perfect<1>(st, a, grid, lds);
}
}  // namespace pmml_tree

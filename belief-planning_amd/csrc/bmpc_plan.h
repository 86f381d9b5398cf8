// bmpc_plan.h -- host-side construction of a plan: scenario-tree topology tables, vector
// layouts and the per-ego workspace layout.  Pure C++ (no HIP), shared by libbmpc.so and
// the test-only host build.
#pragma once

#include <string>
#include <vector>

#include "bmpc_core.h"

namespace bmpc {

struct HostPlan {
  Plan plan;        // pointers in plan.t refer to the vectors below
  Layout lay;
  // topology storage
  std::vector<int32_t> br_depth, br_len, br_ndx, br_ndu, br_child0, br_parent;
  std::vector<int32_t> x_u, x_srcu, x_srcx, x_cone, x_conepos, x_branch, succ_off, succ,
      lvl_off, lvl_nodes, u_x, u_cone, cone_b, cone_i, cone_c, cone_q, cone_off;
  // all tables concatenated (for one device copy) and the offset of each table in it
  std::vector<int32_t> blob;
  std::vector<size_t> blob_off;
  void point_tables(const int32_t* base);   // set plan.t pointers into `base` (blob layout)
};

// Validate `desc` and build everything.  Returns "" on success, else an error message.
std::string build_plan(const bmpc_plan_desc& desc, HostPlan& hp);

}  // namespace bmpc

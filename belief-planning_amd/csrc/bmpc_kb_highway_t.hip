// bmpc_kb_highway_t.hip -- small-batch CVaR IPM kernel (k_solve_blk) of the highway model in transform plans (BMPC_PLAN_TRANSFORM).
// Its own translation unit: BMPC_FLAT_SLAB makes the slab pointers generic, so that the IPM's
// most-visited arrays can live in the workgroup's LDS (bmpc_dev.h, k_solve_blk).
#define BMPC_FLAT_SLAB 1
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_solver_blk_highway_t(const SolveLaunch& a) { return launch_solver_blk<HighwayT, false>(a); }

}  // namespace dev
}  // namespace bmpc

// bmpc_kb_quadruped.hip -- small-batch CVaR IPM kernel (k_solve_blk) of the quadruped model (BMPC_MODEL_QUADRUPED).
// Its own translation unit: BMPC_FLAT_SLAB makes the slab pointers generic, so that the IPM's
// most-visited arrays can live in the workgroup's LDS (bmpc_dev.h, k_solve_blk).
#define BMPC_FLAT_SLAB 1
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_solver_blk_quadruped(const SolveLaunch& a) { return launch_solver_blk<Quadruped, true>(a); }

}  // namespace dev
}  // namespace bmpc

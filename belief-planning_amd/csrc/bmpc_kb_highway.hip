// bmpc_kb_highway.hip -- small-batch CVaR IPM kernel (k_solve_blk) of the highway model (BMPC_MODEL_HIGHWAY).
// Its own translation unit: BMPC_FLAT_SLAB makes the slab pointers generic, so that the IPM's
// most-visited arrays can live in the workgroup's LDS (bmpc_dev.h, k_solve_blk).
#define BMPC_FLAT_SLAB 1
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_solver_blk_highway(const SolveLaunch& a) { return launch_solver_blk<Highway, true>(a); }

}  // namespace dev
}  // namespace bmpc

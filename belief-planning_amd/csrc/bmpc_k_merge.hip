// bmpc_k_merge.hip -- solver kernels of the merge-scene model (BMPC_MODEL_HIGHWAY_MERGE): CVaR IPM with S / Fx / bx.
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_tree_merge(const SolveLaunch& a) { return launch_tree<HighwayMerge>(a); }
hipError_t launch_solver_merge(const SolveLaunch& a) { return launch_solver<HighwayMerge, false>(a); }

}  // namespace dev
}  // namespace bmpc

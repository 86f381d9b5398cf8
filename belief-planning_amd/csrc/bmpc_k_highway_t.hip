// bmpc_k_highway_t.hip -- solver kernels of the highway model in transform plans (BMPC_PLAN_TRANSFORM): CVaR IPM with solve's S / Fx / bx.
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_tree_highway_t(const SolveLaunch& a) { return launch_tree<HighwayT>(a); }
hipError_t launch_solver_highway_t(const SolveLaunch& a) { return launch_solver<HighwayT, false>(a); }

}  // namespace dev
}  // namespace bmpc

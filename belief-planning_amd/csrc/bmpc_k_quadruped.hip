// bmpc_k_quadruped.hip -- solver kernels of the quadruped model (BMPC_MODEL_QUADRUPED): CVaR IPM and the QP controllers.
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_tree_quadruped(const SolveLaunch& a) { return launch_tree<Quadruped>(a); }
hipError_t launch_solver_quadruped(const SolveLaunch& a) { return launch_solver<Quadruped, true>(a); }

}  // namespace dev
}  // namespace bmpc

// bmpc_k_highway.hip -- solver kernels of the highway model (BMPC_MODEL_HIGHWAY): CVaR IPM and the OSQP-class QP controllers.
#include "bmpc_dev.h"

namespace bmpc {
namespace dev {

hipError_t launch_tree_highway(const SolveLaunch& a) { return launch_tree<Highway>(a); }
hipError_t launch_solver_highway(const SolveLaunch& a) { return launch_solver<Highway, true>(a); }
hipError_t launch_loop_highway(const SolveLaunch& a, const bmpc_env_desc& env, int t0, int nsteps, double* scene,
                               double* stats) {
  return launch_loop<Highway>(a, env, t0, nsteps, scene, stats);
}

}  // namespace dev
}  // namespace bmpc

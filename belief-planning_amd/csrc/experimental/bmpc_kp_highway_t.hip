// bmpc_kp_highway_t.hip -- the phase-per-kernel CVaR IPM of the BMPC_MODEL_HIGHWAY with solve's S / Fx / bx model (bmpc_dev_ph.h).
// Every phase function is inlined into the kernel that runs it: no out-of-line device call, so
// no callee-saved-register round trips through scratch.
#define BMPC_INLINE_ALL 1
#include "bmpc_dev_ph.h"

namespace bmpc {
namespace dev {

hipError_t launch_ipm_phased_highway_t(const SolveLaunch& a) { return launch_ipm_phased<HighwayT>(a); }

}  // namespace dev
}  // namespace bmpc

"""CPU oracle for the branch-MPC hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, in plain NumPy/SciPy, the reference algorithm of
Gavinli-lgf/belief-planning for the north-star path:

* ``model``     -- the CasADi SX graphs of ``highway_branch_dyn.PredictiveModel`` and
                   ``quadruped_branch_dyn.PredictiveModel`` (dynamics, Jacobians,
                   obstacle rollouts, branch probabilities and collision linearisation);
* ``tree``      -- ``MPC_branch.BranchTree`` + ``inittree``/``updatetree`` and the dense
                   problem assembly of ``BranchMPC_CVaR`` / ``BranchMPCProx``;
* ``ecos_ipm``  -- a restatement of ECOS' primal-dual homogeneous-embedding IPM
                   (ECOS itself is an un-vendored, un-installed dependency);
* ``qp_ipm``    -- a high-accuracy QP solve standing in for OSQP+polish.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker.  The product path (``belief-planning_amd``)
never imports it and fails loudly when the HIP library is missing.
"""

/*
 * bmpc.h -- C ABI of the MI355X batched branch-MPC library (libbmpc.so).
 *
 * Drop-in boundary for the reference's controller / predictive-model surface
 * (Gavinli-lgf/belief-planning).  Every entry point replaces a reference interface:
 *
 *   bmpc_plan_create   <- BranchMPC_CVaR.__init__      MPC_branch.py:1601-1669
 *                         BranchMPCProx.__init__        MPC_branch.py:84-128
 *                         Init_MPC.initBranchMPC/initquadBranchMPC  Init_MPC.py:40-94
 *                         PredictiveModel.__init__      highway_branch_dyn.py:264-281,
 *                                                       quadruped_branch_dyn.py:155-173
 *   bmpc_set_policies  <- PredictiveModel.update_backup highway_branch_dyn.py:331-334
 *                         (the backup lambdas, traced to descriptors)
 *   bmpc_reset         <- "self.BT is None" first-solve path (inittree) MPC_branch.py:2062-2064
 *   bmpc_solve         <- BranchMPC_CVaR.solve           MPC_branch.py:2043-2092
 *                         BranchMPCProx.solve             MPC_branch.py:384-423
 *                         BranchMPC.solve                 MPC_branch.py:1171-1210
 *                         (BMPC_CTRL_PROX: OSQP QP, status 1 = solved / -2 = not)
 *                         (tree update, linearisation, assembly, ecos.solve / OSQP, unpack)
 *   bmpc_get_tree      <- BranchTree fields + BT2array    MPC_branch.py:65-78,2108-2122
 *   bmpc_get_branch_dp <- BranchTree.dp                    MPC_branch.py:1711,1842
 *   bmpc_set_transform <- solve(..., S, bx) arguments      MPC_branch.py:2043-2057
 *   bmpc_set_fx        <- solve(..., Fx) argument          MPC_branch.py:2055-2056
 *   bmpc_model_eval    <- PredictiveModel.dyn_linearization / branch_eval / zpred_eval /
 *                         col_eval                         highway_branch_dyn.py:284-325
 *   bmpc_model_eval_ref<- the same of PredictiveModel_merge with psiref backups
 *                                                          highway_branch_dyn.py:54-130,400-502
 *   bmpc_set_lane_ref  <- PredictiveModel_merge(..., merge_ref) / the refpsi interpolant of
 *                         the psiref backups              main_branch.py:78-85
 *   bmpc_env_step      <- Highway_env.step + Highway_sim collision rule
 *                                                          Highway_env_branch.py:83-184,421-429
 *
 * Conventions: all host buffers are caller-owned, C-contiguous, ego-major, float64
 * (int32 for status/iteration counts).  Return codes are 0 on success and a negative
 * errno-style code on failure; bmpc_last_error() gives a thread-local message.  A plan
 * owns its device buffers and the per-ego persistent warm-start state; calls are
 * synchronous on the plan's HIP stream unless the *_device variant is used.
 * Per-ego status follows ECOS exit codes for the CVaR controller (>= 0 means
 * "feasible", MPC_branch.py:2141) and OSQP status_val for the QP controllers
 * (1 means "feasible", MPC_branch.py:482).  CVaR status -9 is not an ECOS code: the
 * kernel's internal consistency guard on its best-iterate state tripped (never expected).
 */
#ifndef BMPC_H
#define BMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BMPC_ABI_VERSION 2

#define BMPC_MAX_N 8      /* state dimension            */
#define BMPC_MAX_D 4      /* input dimension            */
#define BMPC_MAX_FX 8     /* rows of Fx                 */
#define BMPC_MAX_FU 8     /* rows of Fu                 */
#define BMPC_MAX_M 4      /* backup policies per branch */

/* controller kinds */
enum {
  BMPC_CTRL_CVAR = 0, /* BranchMPC_CVaR  (ECOS SOCP)   MPC_branch.py:1598 */
  BMPC_CTRL_PROX = 1, /* BranchMPCProx   (OSQP QP)     MPC_branch.py:82   */
  BMPC_CTRL_QP = 2,   /* BranchMPC, active definition (OSQP QP) MPC_branch.py:881 */
  BMPC_CTRL_ROBUST = 3 /* robustMPC: one input sequence against every obstacle prediction
                          of the tree (OSQP QP) MPC_branch.py:1275.  T = N*NB+2 states,
                          U = N*NB+1 inputs, no branch weights; status 1 = solved, the
                          solution is taken whatever the status (:1459) */
};

/* predictive models */
enum {
  BMPC_MODEL_HIGHWAY = 0,       /* highway_branch_dyn.PredictiveModel   */
  BMPC_MODEL_QUADRUPED = 1,     /* quadruped_branch_dyn.PredictiveModel */
  BMPC_MODEL_HIGHWAY_MERGE = 2  /* highway_branch_dyn.PredictiveModel_merge (:400-502) without
                                   psiref policies: BF_traj = softmin_5 of veh_col(obs, ego,
                                   [L+1, W+0.2]) only (:463-467); plans of this model accept a
                                   per-ego state transformation S and state bound bx
                                   (bmpc_set_transform) -- the merge scene's controller */
};

/* backup-policy kinds (what the traced lambdas lower to) */
enum {
  BMPC_POL_MAINTAIN = 0,        /* backup_maintain(x,cons)          p = {Kpsi}          */
  BMPC_POL_BRAKE = 1,           /* backup_brake(x,cons)             p = {Kpsi}          */
  BMPC_POL_LC = 2,              /* backup_lc(x,x0)                  p = x0[0..3]        */
  BMPC_POL_MAINTAIN_TRACKV = 3, /* backup_maintain_trackV(x,cons,v0) p = {Kpsi, v0}     */
  BMPC_POL_FORWARD = 4,         /* quadruped backup_forward(x,v0)   p = {v0}            */
  BMPC_POL_STOP = 5,            /* quadruped backup_stop(x)                             */
  /* the merge ramp's lane-reference tracking backups: the same policies with the psiref
   * argument, psiref(X) = the plan's lane reference (bmpc_set_lane_ref; bmpc_model_eval_ref),
   * a 1-D linear interpolant (casadi.interpolant 'linear', main_branch.py:78-82);
   * highway_branch_dyn.py:54-130 MX branches.  HIGHWAY_MERGE plans only.                 */
  BMPC_POL_MAINTAIN_PSIREF = 6,        /* u = [0, psiref(X) - Kpsi psi]            p = {Kpsi}     */
  BMPC_POL_MAINTAIN_TRACKV_PSIREF = 7, /* u = [0.5 (v0 - v), psiref(X) - Kpsi psi] p = {Kpsi, v0} */
  BMPC_POL_BRAKE_PSIREF = 8            /* u = [softmax([-5, -v], 3), psiref(X) - Kpsi psi]  p = {Kpsi} */
};

/* largest lane reference (grid points) a plan or bmpc_model_eval_ref takes */
#define BMPC_MAX_LANE_REF 4096

typedef struct {
  int32_t kind;
  int32_t reserved;
  double p[4];
} bmpc_policy;

/* POD description of one controller + predictive model (one plan = one batch of egos
 * that share it).  Matrices are row-major with the leading dimension equal to their
 * logical size (Q is n*n, Fx is nFx*n, Fu is nFu*d, ...). */
typedef struct {
  int32_t controller;   /* BMPC_CTRL_*                                   */
  int32_t model;        /* BMPC_MODEL_*                                  */
  int32_t n, d;         /* state / input dimension                      */
  int32_t N, NB, m;     /* steps per branch, branching depth, policies  */
  int32_t nFx, nFu;     /* rows of Fx, Fu                                */
  int32_t maxit;        /* IPM iterations (ECOS default 100)            */
  double dt;
  double ralpha;        /* CVaR alpha (BranchMPC_CVaR ralpha)            */
  double Q[BMPC_MAX_N * BMPC_MAX_N];
  double R[BMPC_MAX_D * BMPC_MAX_D];
  double Qf[BMPC_MAX_N * BMPC_MAX_N];
  double dR[BMPC_MAX_D];
  double Fx[BMPC_MAX_FX * BMPC_MAX_N];
  double bx[BMPC_MAX_FX];
  double Fu[BMPC_MAX_FU * BMPC_MAX_D];
  double bu[BMPC_MAX_FU];
  double Qslack[2];
  /* model constants:
   *   highway   {L, W, s1, N_lane}          (Branch_constants + PredictiveModel ctor)
   *   quadruped {L1, W1, L2, W2, col_tol, s1} (Quad_constants)                       */
  double mc[8];
  double feastol, abstol, reltol; /* ECOS tolerances (defaults 1e-8)              */
  int32_t flags;        /* BMPC_PLAN_* (ABI 2)                            */
  int32_t reserved_flags;
} bmpc_plan_desc;

/* plan flags */
enum {
  BMPC_PLAN_TRANSFORM = 1  /* CVaR plans of the HIGHWAY model that accept the per-solve S / Fx / bx
                              arguments of BranchMPC_CVaR.solve (bmpc_set_transform, bmpc_set_fx);
                              HIGHWAY_MERGE plans always do */
};

typedef struct bmpc_ctx bmpc_ctx;
typedef struct bmpc_plan bmpc_plan;

/* plan geometry returned by bmpc_plan_info (all int32) */
enum {
  BMPC_INFO_T = 0,      /* totalx  (state nodes)                 */
  BMPC_INFO_U,          /* totalu  (input nodes)                 */
  BMPC_INFO_BDIM,       /* non-leaf branches                     */
  BMPC_INFO_NBRANCH,    /* branches incl. root                   */
  BMPC_INFO_NV,         /* primal variables of the solver vector */
  BMPC_INFO_NEQ,        /* equality rows                         */
  BMPC_INFO_NROWS,      /* conic rows (LP + SOC)                 */
  BMPC_INFO_NCONES,     /* second-order cones                    */
  BMPC_INFO_LP,         /* LP rows (dims['l'])                   */
  BMPC_INFO_BATCH,
  BMPC_INFO_WS_DOUBLES, /* per-ego HBM workspace slab (doubles)  */
  BMPC_INFO_SOLVER,     /* solver kernel of the plan's last solve (BMPC_KERNEL_*)      */
  BMPC_INFO_COUNT
};

/* solver kernels (BMPC_INFO_SOLVER): which launch path the last solve took */
enum {
  BMPC_KERNEL_NONE = 0,      /* no solve yet                                              */
  BMPC_KERNEL_IPM_RICH = 1,  /* k_ipm, one wave per ego, topology + coupling system in LDS */
  BMPC_KERNEL_IPM_LEAN = 2,  /* k_ipm, one wave per ego, coupling system in the slab       */
  BMPC_KERNEL_IPM_BLK4 = 3,  /* k_solve_blk, one ego per 4-wave workgroup (small batches)  */
  BMPC_KERNEL_IPM_BLK8 = 4,  /* k_solve_blk, one ego per 8-wave workgroup (small batches)  */
  BMPC_KERNEL_QP_RICH = 5,   /* k_qp (OSQP-class controllers), LDS-rich                    */
  BMPC_KERNEL_QP_LEAN = 6,   /* k_qp, lean                                                 */
  BMPC_KERNEL_LOOP_RICH = 7, /* k_loop (bmpc_loop_device): env + tree + IPM steps per ego    */
  BMPC_KERNEL_LOOP_LEAN = 8  /* k_loop, lean                                                 */
};

const char* bmpc_last_error(void);
int bmpc_abi_version(void);

int bmpc_open(int hip_device, bmpc_ctx** out);
int bmpc_close(bmpc_ctx* ctx);

int bmpc_plan_create(bmpc_ctx* ctx, const bmpc_plan_desc* desc, int batch, bmpc_plan** out);
int bmpc_plan_destroy(bmpc_plan* plan);
int bmpc_plan_info(const bmpc_plan* plan, int32_t* info /* [BMPC_INFO_COUNT] */);

/* update_backup: policies[batch][m]; mask[batch] (NULL = all egos) */
int bmpc_set_policies(bmpc_plan* plan, const bmpc_policy* policies, const uint8_t* mask);
/* the policies in force [batch][m], including the device-side lane-change re-targets of
 * bmpc_env_step (update_backup, Highway_env_branch.py:117-118) */
int bmpc_get_policies(bmpc_plan* plan, bmpc_policy* policies);
/* forget the warm start (next solve runs inittree); mask NULL = all egos */
int bmpc_reset(bmpc_plan* plan, const uint8_t* mask);

/* One controller solve for every ego of the plan (host buffers).
 *   x, z, xref : [batch][n]
 *   upred      : [batch][U][d]     xpred : [batch][T][n]
 *   branch_w   : [batch][nbranch-1] (BFS order of BT2array)
 *   J          : [batch]            objective (CVaR: the J variable; QP: cost)
 *   status     : [batch]            ECOS exitFlag / OSQP status_val
 *   iters      : [batch]
 * Any output pointer may be NULL. */
int bmpc_solve(bmpc_plan* plan, const double* x, const double* z, const double* xref,
               double* upred, double* xpred, double* branch_w, double* J,
               int32_t* status, int32_t* iters);

/* Same with device pointers, enqueued on `stream` (hipStream_t, NULL = plan stream),
 * no host synchronisation. */
int bmpc_solve_device(bmpc_plan* plan, const double* d_x, const double* d_z,
                      const double* d_xref, double* d_upred, double* d_xpred,
                      double* d_branch_w, double* d_J, int32_t* d_status,
                      int32_t* d_iters, void* stream);

/* Checkpoint / resume of the per-ego warm start: the state the reference keeps
 * in the controller object between solves -- uLin [batch][U+1][d] (shifted by updatetree,
 * MPC_branch.py:1813-1823), the previous branch probabilities p [batch][bdim][m] (argmax
 * child, :1818), the frozen Jcons [batch] (CVaR, :1939) and OldInput [batch][d] (the rate
 * cost of BranchMPCProx, :311,:421).  set marks the egos as initialised (the next solve runs
 * updatetree, not inittree); NULL p / jcons / old_input keep the current values; mask NULL
 * = all egos. */
int bmpc_get_warm_start(bmpc_plan* plan, double* uLin, double* p, double* jcons, double* old_input);
/* robustMPC's warm start: the linearisation trajectory xLin [batch][T][n] and uLin
 * [batch][U][d] (the previous prediction shifted by one step, MPC_branch.py:1429-1431) and
 * OldInput [batch][d]; set marks the egos initialised; get/set NULL pointers skip. */
int bmpc_get_robust_warm_start(bmpc_plan* plan, double* xLin, double* uLin, double* old_input);
int bmpc_set_robust_warm_start(bmpc_plan* plan, const double* xLin, const double* uLin,
                               const double* old_input, const uint8_t* mask);
int bmpc_set_warm_start(bmpc_plan* plan, const double* uLin, const double* p,
                        const double* jcons, const double* old_input, const uint8_t* mask);

/* Per-ego state transformation S and state bound bx of the next solves: the S / bx arguments
 * of BranchMPC_CVaR.solve(x, z, xRef, S, Fx, bx) (MPC_branch.py:2043-2057), used by the merge
 * scene (Highway_env_branch.py:358-367).  HIGHWAY_MERGE plans and HIGHWAY CVaR plans created
 * with BMPC_PLAN_TRANSFORM.
 *   S    [batch][n][n] row-major, or NULL = S is None for every ego (the reference resets
 *        self.S on every solve, so pass it before each solve);
 *   s_on [batch] (NULL = 1 for all egos when S is given): 0 marks "S is None" for that ego;
 *   bx   [batch][nFx], or NULL = keep the current bound (the reference keeps self.bx).
 * The state rows follow the reference's build / update split exactly: the first solve
 * (buildIneqConstr :1894-1901) writes Fx S x <= bx (Fx x <= bx without S) from the current
 * Fx and bx; a later solve rewrites them only when S is on (updateIneqConstr :2025-2036), and
 * then also pushes the collision row's dh[0] to sign(dh0) max(0.1, |dh0|) while its rhs keeps
 * the unclipped h0; with S off the rows and their bound keep their last values (:2016-2024
 * patch the collision row alone).  The cones' middle rows use W1 S (W1 without S) on every
 * solve (:1935-1937, :1995-1998).  mask NULL = all egos. */
int bmpc_set_transform(bmpc_plan* plan, const double* S, const uint8_t* s_on, const double* bx,
                       const uint8_t* mask);
/* Per-ego state-constraint matrix Fx [batch][nFx][n] of the next solves: the Fx argument of
 * BranchMPC_CVaR.solve (self.Fx = Fx, kept until the next one, MPC_branch.py:2055-2056).  It
 * enters the state rows under the rule of bmpc_set_transform (first solve, or S on).  Same
 * plans as bmpc_set_transform; the row count must stay nFx.  mask NULL = all egos. */
int bmpc_set_fx(bmpc_plan* plan, const double* Fx, const uint8_t* mask);

/* Tree of the last solve (host copies; NULL skips):
 *   xbar,zbar [batch][T][n]  ubar [batch][U][d]  w [batch][nbranch]
 *   p [batch][bdim][m]       sol [batch][nv]   (full primal vector, reference layout) */
int bmpc_get_tree(bmpc_plan* plan, double* xbar, double* ubar, double* zbar, double* w,
                  double* p, double* sol);
/* dp = d p / d x of every non-leaf branch of the last solve, [batch][bdim][m][n]: the
 * BranchTree.dp that inittree / updatetree set from branch_eval (MPC_branch.py:1711,1842). */
int bmpc_get_branch_dp(bmpc_plan* plan, double* dp);

/* Average device time per call of each kernel over the solves since the last call
 * (HIP events on the launch stream); ms[0] = tree/linearisation kernel, ms[1] = IPM
 * kernel, count = number of solves timed.  Timing must be enabled first.  Timed solves do
 * not synchronise the host: events are read back every 32 solves and by bmpc_timing. */
int bmpc_enable_timing(bmpc_plan* plan, int on);
int bmpc_timing(bmpc_plan* plan, double* ms /* [2] */, int32_t* count);

/* Per-ego phase cycle counters [batch][24] (s_memtime cycles accumulated since plan
 * creation: tree, residuals, scaling, factor, coupling, kkt, tree-solve, refine, -, init,
 * total, kkt-solve count).  All zero unless the library was built with -DBMPC_PROFILE. */
int bmpc_get_counters(bmpc_plan* plan, double* out);

/* Batched model evaluation at B independent points (parity entry for the model
 * functions).  policies [B][m].  Outputs (NULL skips):
 *   A [B][n][n], Bm [B][n][d], C [B][n], xp [B][n]    at (x, u)
 *   p [B][m], dp [B][m][n]                            branch_eval(x, z)
 *   zpred [B][N][m*n]                                 zpred_eval(z)
 *   h0 [B], dh [B][n]                                 col_eval(x, z) */
int bmpc_model_eval(bmpc_ctx* ctx, const bmpc_plan_desc* desc, const bmpc_policy* policies,
                    int B, const double* x, const double* u, const double* z,
                    double* A, double* Bm, double* C, double* xp, double* p, double* dp,
                    double* zpred, double* h0, double* dh);

/* bmpc_model_eval for models whose policies track a lane reference (BMPC_POL_*_PSIREF):
 * the reference psiref(X) is the linear interpolant of values [nref] over the increasing grid
 * [nref] (2 <= nref <= BMPC_MAX_LANE_REF; outside the grid the end cells extend linearly, as
 * casadi.interpolant 'linear' does).  Replaces PredictiveModel_merge's MX graphs with psiref
 * backups (highway_branch_dyn.py:400-502; the merge scene's pred_model[1], main_branch.py:85,
 * whose zpred_eval the scene calls, Highway_env_branch.py:331).  nref = 0: no reference (then
 * no policy may be a *_PSIREF kind). */
int bmpc_model_eval_ref(bmpc_ctx* ctx, const bmpc_plan_desc* desc, const bmpc_policy* policies,
                        int nref, const double* grid, const double* values,
                        int B, const double* x, const double* u, const double* z,
                        double* A, double* Bm, double* C, double* xp, double* p, double* dp,
                        double* zpred, double* h0, double* dh);

/* The lane reference of a HIGHWAY_MERGE plan's *_PSIREF policies (same form as
 * bmpc_model_eval_ref): shared by every ego of the plan, kept until the next call. */
int bmpc_set_lane_ref(bmpc_plan* plan, int nref, const double* grid, const double* values);

/* Closed-loop sim_overtake scene on the device, one scene per ego of a highway plan:
 * replaces Highway_env_branch.Highway_env.step (Highway_env_branch.py:83-184) around the
 * solve and the collision rule of Highway_sim (:421-429).  */
#define BMPC_ENV_STRIDE 16  /* doubles of per-ego scene state  */
#define BMPC_ENV_NSTAT 8    /* doubles of per-ego statistics   */
typedef struct {
  int32_t n_lane;     /* lanes of the env (LB = [W/2, n_lane*3.6 - W/2], :64); 4 in sim_overtake */
  int32_t reserved;
  double L, W, Kpsi;  /* Branch_constants (main_branch.py:37)                        */
  double v0;          /* 20 (Highway_env_branch.py:22)                               */
  double vlen, vwid;  /* vehicle() size 4 x 2.4 (:29), used by the collision test    */
  double target[4];   /* lane-change target of the env's construction-time backup list */
} bmpc_env_desc;

/* One closed-loop step t of every ego (device pointers, enqueued on `stream`):
 *   scene  [batch][BMPC_ENV_STRIDE]  state: ego x[0..3], obstacle z[4..7], the rest zero at
 *                                    t = 0 (the caller writes the initial states);
 *   upred  [batch][U][d]             the last solve's uPred (ignored at t = 0);
 *   J, status, iters [batch]         the last solve's outputs for the statistics (NULL skips);
 *   x, z, xref [batch][4]            out: the next solve's inputs;
 *   stats  [batch][BMPC_ENV_NSTAT]   accumulated {sum J, sum J^2, infeasible, iterations,
 *                                    solves, steps in collision, collided} (NULL skips).
 * The plan's lane-change policies are re-targeted on the device (update_backup, :118). */
int bmpc_env_step(bmpc_plan* plan, const bmpc_env_desc* env, int t, double* d_scene,
                  const double* d_upred, const double* d_J, const int32_t* d_status,
                  const int32_t* d_iters, double* d_x, double* d_z, double* d_xref,
                  double* d_stats, void* stream);

/* nsteps closed-loop steps t0 .. t0+nsteps-1 of every ego, each bmpc_env_step(t) followed by
 * bmpc_solve_device -- the loop main_branch.sim_overtake runs per ego (Highway_sim,
 * Highway_env_branch.py:408-436: env.step -> controller solve, repeated) -- with the same
 * arguments and the same per-ego results, bit for bit.  The egos' loops are independent, so a
 * CVaR plan whose batch takes the one-wave IPM runs them in ONE launch (k_loop: each wave
 * steps its ego through all nsteps without a device-wide boundary between steps, so no step
 * waits for the slowest ego of the previous one); other batches run the two launches per step.
 * d_upred / d_J / d_status / d_iters hold the last solve's outputs on return (the next call's
 * t0 > 0 reads them); d_x / d_z / d_xref the last step's solve inputs.  Highway CVaR / robust
 * plans without transform (the scene's model); -22 otherwise.  An extension of the drop-in ABI
 * for Monte-Carlo closed-loop batches (BASELINE config 5); the reference has no batched loop. */
int bmpc_loop_device(bmpc_plan* plan, const bmpc_env_desc* env, int t0, int nsteps, double* d_scene,
                     double* d_upred, double* d_x, double* d_z, double* d_xref, double* d_J,
                     int32_t* d_status, int32_t* d_iters, double* d_stats, void* stream);

/* HMM belief-augmented linearisation, batched over B points: replaces
 * HMM_backup_dyn.PredictiveModel.regressionAndLinearization (HMM_backup_dyn.py:216-237) of
 * the graph of calc_xp_expr (:238-276).  M agents (1..4), m backups (1..4), nb = 4 + M*m.
 *   hc      [8]           {dt, L, W, ylb, yub, col_alpha, s1, tran_diag} (Branch_constants)
 *   xb      [B][nb]       [x; b stacked column-major] (CasADi reshape, :244)
 *   u       [B][2]        xbackup [B][M*m][4] (row m*i+j: agent i under backup j)
 * Outputs (NULL skips): xbp [B][nb], A [B][nb][nb], Bm [B][nb][2], C [B][nb],
 *   h0 [B][M][m], Jh [B][M][m][nb]   (h0_i = h_i - Jh_i xb, :226-229) */
int bmpc_hmm_eval(bmpc_ctx* ctx, int M, int m, const double* hc, int B, const double* xb, const double* u,
                  const double* xbackup, double* xbp, double* A, double* Bm, double* C, double* h0,
                  double* Jh);

/* Batched convex QP in OSQP's problem form (the solver behind the belief LTV-MPC,
 * PredictiveControllers.MPC.osqp_solve_qp, PredictiveControllers.py:310-340, which the
 * reference hands to OSQP(...).setup(P, q, A, l, u, polish=True).solve()):
 *     minimise 1/2 x'Px + q'x  subject to  l <= A x <= u
 * by a Mehrotra interior-point method on the quasidefinite KKT matrix, band-factored after a
 * reverse Cuthill-McKee ordering, one wave per problem (csrc/bmpc_bandqp.h).  The problems of
 * a batch share one sparsity pattern:
 *   Pp [n+1], Pi [nnzP]      upper triangle of P, CSC (OSQP keeps only the upper triangle)
 *   Ap [n+1], Ai [nnzA]      A (m x n), CSC; row indices increasing within a column
 *   Px [batch][nnzP], Ax [batch][nnzA], q [batch][n], l, u [batch][m]
 * |bound| >= 1e20 is infinite; a row with l == u is an equality; every problem must classify
 * every row alike.  Outputs: x [batch][n]; y [batch][m] (OSQP's dual, P x + q + A'y = 0;
 * NULL skips); status [batch] (1 solved to eps, -2 max_iter reached, -8 numerical failure);
 * iters [batch] (NULL skips); info [4] = {KKT dimension, bandwidth, inequality rows, band
 * entries} (NULL skips).  -22 when the KKT band does not fit the 160 KB LDS window. */
int bmpc_qp_solve(bmpc_ctx* ctx, int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                  const int32_t* Ai, int batch, const double* Px, const double* q, const double* Ax, const double* l,
                  const double* u, int max_iter, double eps, double* x, double* y, int32_t* status, int32_t* iters,
                  int32_t* info);

#ifdef __cplusplus
}
#endif
#endif /* BMPC_H */

/* mppi_rocm.h — C ABI of the MI355X (gfx950) MPPI rollout-and-reduce engine.
 *
 * Drop-in boundary.  The reference (junofficial/mppi_RobotArm) has no FFI: its
 * boundary is the Python method
 *     MPPIControllerForPathTracking.calc_control_input(observed_x)
 *         -> (u0, u_seq, optimal_traj, sampled_traj_list)          control.py:67-152
 * The Python mirror of that class (mppi_robotarm_amd/controller.py) keeps the
 * O(T) host work of control.py:70-78 and :120-152 and calls the entry points
 * below for the O(K*T) work of control.py:81-118 (ctypes stub: INTEGRATION.md).
 *
 * Conventions: plain C types only.  Device buffers are raw device pointers
 * (the Python side holds them as PyTorch-ROCm tensors); `stream` is a
 * hipStream_t passed as void*.  Every call returns 0 on success or a negative
 * MPPI_E_* code; mppi_last_error() returns the message of the calling thread's
 * last failure.  Calls on one context are serialised on its stream; a context
 * is not re-entrant (the reference controller is stateful and single-threaded,
 * control.py:59,65).
 */
#ifndef MPPI_ROCM_H
#define MPPI_ROCM_H

#ifdef __cplusplus
extern "C" {
#endif

#define MPPI_MAX_T 128       /* horizon limit of the device parameter block          */
#define MPPI_SEARCH_LEN 30   /* waypoints per search window, control.py:203           */

#define MPPI_OK 0
#define MPPI_E_ARG -1        /* bad argument (shape, null pointer, range)             */
#define MPPI_E_HIP -2        /* HIP runtime error (message says which call)            */
#define MPPI_E_SINGULAR -3   /* singular Sigma: the reference raises LinAlgError at   */
                             /* control.py:106 (np.linalg.inv)                          */
#define MPPI_E_EXCHANGE -5   /* multi-GPU in-launch exchange: a rank's row missed the poll
                                bound (MPPI_EXCHANGE_TIMEOUT_US, default ~1 s) on some rank of the
                                step; every rank of the step reports it and none applied the
                                update (the nominal is the one before the step)              */
#define MPPI_E_RETRY -6      /* mppi_np_draw_result: the draw generated fewer accepted   */
                             /* polar attempts than it needed (or its look-back gave up);*/
                             /* the output is incomplete and the state is the caller's   */
                             /* (draw on the host instead)                               */
#define MPPI_E_PATH_END -4   /* mppi_dropin_tick: the updated waypoint index reached   */
                             /* the end of the path (control.py:76-78: the reference   */
                             /* prints "[ERROR] ..." and raises IndexError)           */

/* rollout flags */
#define MPPI_FLAG_FUSED_UPDATE 1u  /* last workgroup also runs median filter, u += w_eps, */
                                   /* shift (control.py:122-149) on device                */
#define MPPI_FLAG_EXCHANGE 2u      /* multi-GPU: the launch exchanges the ranks' partial  */
                                   /* rows itself and merges them (mppi_exchange_attach)  */
#define MPPI_FLAG_HOST_OUT 4u      /* with FUSED_UPDATE: the final workgroup also writes   */
                                   /* the shifted nominal to host-mapped memory; read it  */
                                   /* with mppi_wait_outputs (no copy, no stream sync)    */
#define MPPI_IPC_HANDLE_BYTES 64   /* hipIpcMemHandle_t                                    */
#define MPPI_MAX_WORLD 8           /* ranks of one node for the in-launch exchange         */

/* Arm constants.  m1..g: sys_params.py:1-13, read by _F (control.py:11-18,
 * 241-251).  fk_l1/fk_l2: the link lengths the cost's forward kinematics uses,
 * self.l1 = self.l2 = 1 (control.py:55-56, 178-179, 205-206) — kept separate. */
typedef struct {
    double m1, m2, l1, l2, lc1, lc2, g;
    double fk_l1, fk_l2;
} mppi_arm_params;

/* Constructor arguments of MPPIControllerForPathTracking (control.py:21-35)
 * plus the shard geometry of this device. */
typedef struct {
    int K_local;               /* samples simulated on this device                     */
    int T;                     /* horizon_step_T, 1..MPPI_MAX_T                        */
    int K_total;               /* number_of_samples_K over all devices                 */
    int k_offset;              /* global index of this device's first sample            */
    double delta_t;            /* control.py:53                                         */
    double param_lambda;       /* control.py:43                                         */
    double param_alpha;        /* control.py:44; gamma = lambda (1 - alpha), :45        */
    double param_exploration;  /* control.py:42,98                                      */
    double sigma[4];           /* row-major 2x2 noise covariance, control.py:46         */
    double stage_cost_weight[4];
    double terminal_cost_weight[4];
    mppi_arm_params arm;
    int lanes_per_sample;      /* 0 = auto; 1, 2, 4, 8 or 16 lanes of a wave per sample */
    double param_gamma;        /* gamma of the control cost (control.py:106), used as   */
                               /* given; NaN: lambda (1 - alpha) as control.py:45       */
} mppi_config;

typedef struct mppi_ctx mppi_ctx;

/* Fill *cfg with the defaults a C caller should start from before setting its
 * fields: every field zero except param_gamma = NaN (gamma = lambda (1 - alpha),
 * control.py:45) and arm = sys_params.py:1-13 with the cost's kinematics lengths
 * self.l1 = self.l2 = 1 (control.py:55-56).  A config zeroed with memset or
 * `= {0}` instead has gamma = 0 (no control-cost term).  No device call. */
void mppi_config_init(mppi_config *cfg);

/* Context: device scratch (workgroup partial slabs, arrival counter, step
 * parameter block) is allocated here; no call below allocates.  Fails with
 * MPPI_E_SINGULAR for a singular Sigma. */
int mppi_ctx_create(const mppi_config *cfg, int device, void *stream, mppi_ctx **out);
void mppi_ctx_destroy(mppi_ctx *ctx);
const char *mppi_last_error(void);
int mppi_set_stream(mppi_ctx *ctx, void *stream);
int mppi_ctx_info(const mppi_ctx *ctx, int *lanes_per_sample, int *blocks, int *threads_per_block);

/* In-launch hand-off of the workgroup partial rows chosen at creation: *poll = 1
 * for tagged-granule polling (grid co-resident, at most one workgroup per CU),
 * 0 for arrival counters (larger grids, or MPPI_HANDOFF=counter in the
 * environment).  No reference equivalent (the reference reduces in NumPy,
 * control.py:112-118). */
int mppi_ctx_handoff(const mppi_ctx *ctx, int *poll);

/* Per control step inputs (control.py:70-75): observed state x0[4], the search
 * window ref_path[prev:prev+W, 0:4] (W = min(30, N - prev), row-major W x 4),
 * and the nominal control sequence u[T][2] (self.u_prev).  x0 and the window
 * (with its centred search keys) are copied into the context on the host and
 * reach the next launch by value, as a kernel argument (no copy call); u is
 * uploaded with one stream-ordered copy from a pinned staging block.  u may be
 * NULL to keep the device-resident nominal (device closed loop,
 * MPPI_FLAG_FUSED_UPDATE). */
int mppi_set_step_inputs(mppi_ctx *ctx, const double *x0, const double *window, int W,
                         const double *u);

/* The hot path, control.py:81-118, one launch:
 *   noise_dev   fp32 device noise eps[t][k][d] for this device's samples,
 *               layout [T][K_local][2] (time-major: each step is one coalesced row);
 *   S_dev       optional fp64 [K_local] per-sample cost S (control.py:81-109);
 *   partial_dev optional fp64 [2 + 2T] device partial {rho, eta, N[T][2]} with
 *               rho = min S, eta = sum exp(-(S-rho)/lambda), N = sum exp(.) eps —
 *               the operand of the cross-device exchange;
 *   flags       MPPI_FLAG_FUSED_UPDATE: finish the step on device (single device).
 * The weighted noise w_eps = N / eta (control.py:112-118) is left in the
 * context (mppi_get_weighted_noise). */
int mppi_rollout(mppi_ctx *ctx, const float *noise_dev, double *S_dev, double *partial_dev,
                 unsigned flags);

/* Merge n device partials (fp64 [n][2 + 2T], e.g. the all-gather of every
 * rank's partial_dev) with a log-sum-exp rescale into w_eps; with
 * MPPI_FLAG_FUSED_UPDATE also run the update of control.py:122-149 on device. */
int mppi_merge_partials(mppi_ctx *ctx, const double *partials_dev, int n, unsigned flags);

/* In-launch multi-GPU exchange (one process per GPU on one node; the reference
 * is single-process, so this, like mppi_merge_partials, completes
 * control.py:112-118 across devices).  Setup, once per context:
 *   mppi_exchange_handle(ctx, world, h)  allocates this rank's inbox (uncached
 *     device memory, 2 x world partial rows of tagged granules) and writes its
 *     IPC handle (MPPI_IPC_HANDLE_BYTES) to h;
 *   the caller all-gathers the handles over its process group (rank order);
 *   mppi_exchange_attach(ctx, rank, world, handles)  maps every peer's inbox.
 * Then mppi_rollout(..., partial_dev = NULL, MPPI_FLAG_EXCHANGE [| FUSED_UPDATE])
 * on every rank: the launch's final workgroup writes this rank's partial row
 * into every inbox (xGMI stores), polls its own until all world rows of the
 * step arrived, merges them in rank order and (fused) updates the nominal — no
 * collective call or second launch per step.  Every rank must run the same
 * sequence of exchange launches.  A peer that never arrives ends the poll after
 * ~1 s with a timeout that mppi_sync reports. */
int mppi_exchange_handle(mppi_ctx *ctx, int world, void *handle_out);
int mppi_exchange_attach(mppi_ctx *ctx, int rank, int world, const void *handles);

/* D2H (synchronising) reads of the last step's results. */
int mppi_get_weighted_noise(mppi_ctx *ctx, double *w_eps_host /* [T][2] */);
int mppi_get_nominal(mppi_ctx *ctx, double *u_host /* [T][2] */);

/* Trajectory re-roll (control.py:129-145), fp32 states out_dev[K][T][4] for
 * samples [0, K) of this device:  control(t) = base[(t + T - 1) % T]
 *   (+ eps[(t + T - 1) % T][k] if noise_dev != NULL, exploitation split as
 *   control.py:98), i.e. the reference's off-by-one u[t-1] / v[k, t-1].
 * base_u: host fp64 [T][2], or NULL for the nominal uploaded by the last
 * mppi_set_step_inputs (the pre-update u of the sampled re-roll). */
int mppi_rollout_traj(mppi_ctx *ctx, const double *base_u, const float *noise_dev, int K,
                      float *out_dev);

/* sampled_traj_list's host read-back (control.py:135-145 returns fp64; the
 * re-roll writes fp32).  fp32 -> fp64 is exact, so the widening runs on the
 * host: n fp32 values at src_dev are copied chunk by chunk (chunk_floats each,
 * the last three a half, a quarter and an eighth of it) after the work queued
 * on `stream` (the kernel that wrote them), alternating over copy_streams
 * streams of the object's own (0: on `stream` itself), into a page-locked ring
 * of `slots` chunks, and `workers` host threads widen each landed chunk into
 * dst_host (n fp64, any host memory) while the next chunks are in flight.
 * Half the bytes of a device-side widening cross the host link, and the
 * values are the same.  mppi_readback_run returns when dst_host is written. */
typedef struct mppi_readback mppi_readback;
int mppi_readback_create(int device, int workers, int slots, long long chunk_floats, int copy_streams,
                         mppi_readback **out);
void mppi_readback_destroy(mppi_readback *rb);
int mppi_readback_run(mppi_readback *rb, void *stream, const float *src_dev, double *dst_host, long long n);

/* The optimal trajectory of control.py:129-134 (the updated controls u_new
 * before the shift of :148-149, off-by-one u_new[t-1]) after a launch with
 * MPPI_FLAG_FUSED_UPDATE: fp32 states out_dev[T][4] of one re-roll from x0,
 * the controls taken from the update itself (no host round trip).
 * MPPI_E_ARG before the first fused update. */
int mppi_optimal_traj(mppi_ctx *ctx, float *out_dev);

/* One synchronising read-back of a fused control step: the shifted nominal
 * u[T][2] fp64 (the new self.u_prev, control.py:148-149) into u_host and, if
 * traj_dev is not NULL, the fp32 [T][4] trajectory it holds into traj_host. */
int mppi_get_step_outputs(mppi_ctx *ctx, double *u_host, const float *traj_dev, float *traj_host);

/* The optimal trajectory of control.py:129-134 on the host in fp64 from the
 * updated controls u_new[T][2] (before the shift): x_{t+1} = _F(x_t, u_new[t-1])
 * from x0[4], _F as control.py:234-263 (the context's arm constants and
 * delta_t).  O(T) host work; traj_out[T][4] fp64. */
int mppi_optimal_traj_host(const mppi_ctx *ctx, const double *x0, const double *u_new, double *traj_out);

/* Wait for the last MPPI_FLAG_HOST_OUT launch (mppi_rollout or
 * mppi_merge_partials) to publish its outputs (a spin on a host-mapped flag
 * word), then return the shifted nominal u_out[T][2] fp64 and, if traj_out is
 * not NULL, the fp64 optimal trajectory from x0 (as mppi_optimal_traj_host on
 * the update's u_new). */
int mppi_wait_outputs(mppi_ctx *ctx, const double *x0, double *u_out, double *traj_out);

/* The whole single-device control step of calc_control_input (control.py:81-152)
 * in one call, for the drop-in: stage x0, the window and the nominal u[T][2]
 * (NULL: keep the device-resident one), launch the fused rollout + update on
 * noise_dev ([T][K_local][2] fp32; S_dev nullable), wait until the launch's final
 * workgroup has written the shifted nominal to coherent host-mapped memory (a
 * spin on its flag word: no copy, no stream synchronise), return it in
 * u_out[T][2] fp64 (the new self.u_prev), and, if traj_out is not NULL, the
 * optimal trajectory of control.py:129-134 (off-by-one u_new[t-1]) in fp64
 * computed on the host from the update (O(T): one re-roll of _F,
 * control.py:234-263, in fp64 like the reference).  If next_noise_dev is not
 * NULL, the next step's Philox noise (seed, next_step) is queued into it right
 * after the rollout launch (stream-ordered behind it: the draw runs once the
 * rollout has read noise_dev, which may be the same buffer), so it overlaps the
 * host's remaining work and the caller's.  Needs T >= 5
 * (device median filter).  With an exchange attached (mppi_exchange_attach) the
 * launch also trades and merges every rank's partial row (MPPI_FLAG_EXCHANGE),
 * so one call per rank is one multi-GPU control step; every rank must then make
 * the same sequence of calls. */
int mppi_step_dropin(mppi_ctx *ctx, const double *x0, const double *window, int W, const double *u,
                     const float *noise_dev, double *S_dev, float *next_noise_dev, unsigned long long seed,
                     unsigned long long next_step, double *u_out, double *traj_out);

/* The drop-in's host buffers, bound once (mppi_dropin_bind) so that a control
 * step is one call with no arguments to convert (mppi_dropin_tick):
 *   path, rows, stride  the caller's ref_path (rows of fp64 `stride` apart,
 *                       columns x, y, dq1, dq2 first — run.py's
 *                       ref_path[:, 0:4] view is one; read at every tick, so
 *                       in-place edits are seen as the reference sees them);
 *   fk_l1, fk_l2        self.l1, self.l2 of _get_nearest_waypoint (control.py:
 *                       205-206);
 *   x0                  observed_x (4 fp64), read at every tick;
 *   idx                 [0] self.prev_waypoints_idx, in and out; [1] out: its
 *                       value before the tick (the "prev_idx" print);
 *   u                   self.u_prev (T x 2 fp64): read as this tick's nominal,
 *                       then overwritten with the shifted nominal (the aliasing
 *                       return of control.py:152);
 *   traj                the optimal trajectory (T x 4 fp64) out, or NULL;
 *   noise_dev, next_noise_dev, S_dev, seed: as mppi_step_dropin. */
typedef struct {
    const double *path;
    int rows, stride;
    double fk_l1, fk_l2;
    const double *x0;
    long long *idx;
    double *u;
    double *traj;
    const float *noise_dev;
    float *next_noise_dev;
    double *S_dev;
    unsigned long long seed;
} mppi_dropin_binding;

int mppi_dropin_bind(mppi_ctx *ctx, const mppi_dropin_binding *b);

/* One calc_control_input (control.py:67-152) on the bound buffers: the fp64
 * nearest-waypoint update of control.py:70-74 (_get_nearest_waypoint, :200-232:
 * forward kinematics, first-occurrence argmin of ((x - rx)^2 + (y - ry)^2) * 100
 * over ref_path[prev : prev + 30], the same fp64 operations), then
 * MPPI_E_PATH_END without launching anything if the new index is at the end of
 * the path (control.py:76-78), else mppi_step_dropin on the window
 * ref_path[idx : idx + 30] with the next step's noise (seed, next_step). */
int mppi_dropin_tick(mppi_ctx *ctx, unsigned long long next_step);

/* mppi_dropin_tick in two halves, so the caller can do host work while the
 * launch runs (the drop-in allocates the call's fresh sampled_traj_list,
 * control.py:135, in between): _launch does everything up to and including the
 * launch (MPPI_E_PATH_END as mppi_dropin_tick, nothing launched); _wait waits
 * for the published outputs and writes u and traj.  Every successful _launch
 * must be followed by one _wait before the next _launch. */
int mppi_dropin_tick_launch(mppi_ctx *ctx, unsigned long long next_step);
int mppi_dropin_tick_wait(mppi_ctx *ctx);

/* Counter-based Philox4x32-10 Gaussian noise with covariance Sigma (replaces
 * np.random.multivariate_normal, control.py:163, for device-resident runs; not
 * bit-equal to NumPy).  Values depend only on (seed, step, t, global k), so a
 * shard generates exactly its slice of the unsharded draw.  Layout [T][K_local][2]. */
int mppi_noise_philox(mppi_ctx *ctx, unsigned long long seed, unsigned long long step,
                      float *out_dev);

/* Wait for the context stream.  MPPI_E_HIP if a bounded in-launch spin of the
 * granule hand-off gave up since the last check (that launch's results are
 * invalid; it cannot happen while the grid is co-resident). */
int mppi_sync(mppi_ctx *ctx);

/* Diagnostics: in a -DMPPI_STAMPS build the rollout kernel writes a per-workgroup
 * timeline (16 uint64 per workgroup) to dbg_dev; product builds ignore it. */
int mppi_debug_set_buffer(mppi_ctx *ctx, void *dbg_dev);

/* Diagnostics: host-side phase ends (microseconds from entry) of the last
 * mppi_step_dropin: [0] inputs staged, [1] rollout launched, [2] next noise
 * queued, [3] the rollout's outputs seen in host memory, [4] outputs copied +
 * trajectory. */
int mppi_debug_dropin_times(const mppi_ctx *ctx, double *us_out);

/* Tests: the nearest window slot of the first K samples at every step, as the
 * rollout evaluates it (_get_nearest_waypoint inside _c, control.py:176-180 and
 * :205-215): the same fp32 dynamics and packed argmin on the current step
 * inputs and noise_dev ([T][K_local][2] fp32).  slot_dev[K][T] (int32 device)
 * receives the window slot (0-based, relative to prev_waypoints_idx) and
 * pos_dev[K][T][2] (fp32 device) the end-effector position it was searched for. */
int mppi_debug_nearest(mppi_ctx *ctx, const float *noise_dev, int K, int *slot_dev, float *pos_dev);

/* ------------------------------------------------------------------------
 * n-link planar chain (BASELINE config 5: "7-DoF arm dynamics (extended
 * sys_params.py), K=131072 T=128, xydq_circle.txt reference").  The reference
 * has no such model; it is BUILD-DEFINED (oracle/chain_oracle.py: mass matrix
 * D_ab = mu_ab cos(th_a - th_b) + delta_ab I_a in absolute angles plus the joint
 * armature J, Coriolis, gravity, joint damping b, Cholesky solve, semi-implicit
 * Euler as control.py:256-259) and reduces to the reference _F
 * (control.py:234-263) at n = 2 with I = l and J = b = 0.  The
 * cost is control.py:174-232 on (end-effector x, y, dq_1, dq_2).  Same
 * conventions as above; noise is [T][K_local][n] fp32, u and w_eps are T x n
 * row-major, x0 = [q(n), dq(n)].
 * ------------------------------------------------------------------------ */
#define MPPI_CHAIN_MAX_DOF 8   /* array capacity; n in [2, 7] is supported */

typedef struct {
    int n;                                  /* links, 2..7                                */
    double m[MPPI_CHAIN_MAX_DOF];           /* masses                                     */
    double l[MPPI_CHAIN_MAX_DOF];           /* lengths (dynamics)                         */
    double lc[MPPI_CHAIN_MAX_DOF];          /* joint-to-centre-of-mass distances          */
    double I[MPPI_CHAIN_MAX_DOF];           /* inertias about the centre of mass          */
    double fk[MPPI_CHAIN_MAX_DOF];          /* lengths used by the cost's kinematics      */
    double J[MPPI_CHAIN_MAX_DOF];           /* joint armature (rotor inertia)             */
    double b[MPPI_CHAIN_MAX_DOF];           /* joint viscous damping                      */
    double g;
} mppi_chain_params;

typedef struct {
    int K_local, T, K_total, k_offset;      /* as mppi_config                             */
    double delta_t, param_lambda, param_alpha, param_exploration;
    double sigma[MPPI_CHAIN_MAX_DOF * MPPI_CHAIN_MAX_DOF]; /* n x n row-major, SPD        */
    double stage_cost_weight[4];            /* on (x, y, dq_1, dq_2), control.py:185      */
    double terminal_cost_weight[4];         /* control.py:198                             */
    mppi_chain_params chain;
    int precision;                          /* rollout arithmetic: 0 fp32 (default), 1 fp64
                                               (for spread weights: see DESIGN §3b)       */
    int lanes_per_sample;                   /* 0 = auto; 1, or 4 (fp32: a quad per sample,
                                               lane p the link pair (2p, 2p+1))           */
    double param_gamma;                     /* as mppi_config.param_gamma: control.py:45's
                                               gamma as given; NaN = lambda (1 - alpha)  */
} mppi_chain_config;

typedef struct mppi_chain_ctx mppi_chain_ctx;

/* As mppi_config_init for the chain: every field zero except param_gamma = NaN
 * (lambda (1 - alpha)) and chain.g = 9.81 (sys_params.py:13); the caller sets n,
 * the link parameters, Sigma and the rest.  No device call. */
void mppi_chain_config_init(mppi_chain_config *cfg);

/* control.py:21-65 with the chain model; MPPI_E_SINGULAR if Sigma is not SPD. */
int mppi_chain_ctx_create(const mppi_chain_config *cfg, int device, void *stream, mppi_chain_ctx **out);
void mppi_chain_ctx_destroy(mppi_chain_ctx *ctx);
int mppi_chain_set_stream(mppi_chain_ctx *ctx, void *stream);
int mppi_chain_ctx_info(const mppi_chain_ctx *ctx, int *blocks, int *threads_per_block, int *poll,
                        int *lanes_per_sample);
/* inputs of control.py:70-75: x0[2n], the window (W x 4), u[T*n] (NULL: keep the device nominal) */
int mppi_chain_set_step_inputs(mppi_chain_ctx *ctx, const double *x0, const double *window, int W,
                               const double *u);
/* control.py:81-118 (+ :122-149 with MPPI_FLAG_FUSED_UPDATE) for the chain */
int mppi_chain_rollout(mppi_chain_ctx *ctx, const float *noise_dev, double *S_dev, double *partial_dev,
                       unsigned flags);
int mppi_chain_merge_partials(mppi_chain_ctx *ctx, const double *partials_dev, int n, unsigned flags);
/* In-launch exchange for the chain (as mppi_exchange_handle / _attach; rows of
 * 2 + nT values). */
int mppi_chain_exchange_handle(mppi_chain_ctx *ctx, int world, void *handle_out);
int mppi_chain_exchange_attach(mppi_chain_ctx *ctx, int rank, int world, const void *handles);
int mppi_chain_get_weighted_noise(mppi_chain_ctx *ctx, double *w_eps_host);
int mppi_chain_get_nominal(mppi_chain_ctx *ctx, double *u_host);
/* After a MPPI_FLAG_FUSED_UPDATE launch (control.py:120-149 on the device): the
 * shifted nominal u_out[T][n] (the drop-in's returned sequence) and, when traj_out
 * is given, the optimal trajectory of control.py:129-134 in fp64 on the host from
 * x0[2n] and the update before its shift, traj_out[T][2n] (q, dq).  Replaces the
 * read-back of w_eps + the host median + u += w_eps + the trajectory launch.
 * With MPPI_FLAG_HOST_OUT on that launch, the chain queues this read-back right
 * behind it, so work queued afterwards (the next noise) does not delay the wait. */
int mppi_chain_wait_outputs(mppi_chain_ctx *ctx, const double *x0, double *u_out, double *traj_out);
/* The spread of the last step's weights (control.py:297-314): eta = sum_k
 * exp(-(S_k - min S) / lambda) of the update read by mppi_chain_wait_outputs or
 * the weighted noise read by mppi_chain_get_weighted_noise (NaN before either);
 * eta >= 1, and eta - 1 is the weight outside the best sample (0: one-hot).
 * ChainMPPIController's precision="auto" re-runs a step in fp64 when it exceeds
 * 1e-6. */
int mppi_chain_last_eta(const mppi_chain_ctx *ctx, double *eta);
/* control.py:129-134 for the chain on the host in fp64: traj_out[T][2n] from x0[2n]
 * and the updated (not yet shifted) controls u_new[T][n]. */
int mppi_chain_optimal_traj_host(mppi_chain_ctx *ctx, const double *x0, const double *u_new, double *traj_out);
/* control.py:129-145 analogue: out_dev[K][T][2n] fp32 (q, dq) */
int mppi_chain_rollout_traj(mppi_chain_ctx *ctx, const double *base_u, const float *noise_dev, int K,
                            float *out_dev);
/* N(0, Sigma) noise [T][K_local][n] from Philox4x32-10 (global sample index: shard-invariant) */
int mppi_chain_noise_philox(mppi_chain_ctx *ctx, unsigned long long seed, unsigned long long step,
                            float *out_dev);
int mppi_chain_sync(mppi_chain_ctx *ctx);
int mppi_chain_debug_set_buffer(mppi_chain_ctx *ctx, void *dbg_dev);
/* Tests only: one rollout (as mppi_chain_rollout with no flags; S_dev nullable)
 * through a build of the same kernel that also records the window slot every
 * sample picked at every step (the argmin of control.py:205-215 inside _c),
 * slots_dev int32 [K_local][T].  7-link contexts only.  The parity tests use it
 * to recompute a sample's fp64 cost with the device's own picks. */
int mppi_chain_debug_slots(mppi_chain_ctx *ctx, const float *noise_dev, double *S_dev, int *slots_dev);

/* ------------------------------------------------------------------------
 * The reference's own noise on the device: NumPy's legacy global-RNG stream of
 * np.random.multivariate_normal(mu, Sigma, (K, T)) (control.py:154-164), the
 * drop-in's default noise="numpy", generated bit for bit — the same values
 * and the same RNG state left behind as NumPy's draw — when Sigma's transform
 * is a scaled column permutation (run.py's 20 I, the chain's diagonal Sigma;
 * mppi_robotarm_amd/hostrng.py monomial_transform).  Replaces the host draw
 * (hostrng / np_legacy_gauss.c) and the upload of its 67 MB at config 3.
 *
 * Host inputs the device cannot make: the MT19937 jump polynomials x^J mod P
 * (np_legacy_gauss.c mppi_np_jump_poly) and glibc's log constants, read from
 * the process's libm and checked against its log() (mppi_np_log_params).
 * ------------------------------------------------------------------------ */
#define MPPI_NP_POLY_WORDS 312          /* 64-bit words of a jump polynomial (degree < 19937) */
#define MPPI_NP_LOG_DATA 274            /* doubles of the log constants (np_glibc_log.h)       */
#define MPPI_NP_MAX_DU 8                /* components per step                                 */
#define MPPI_NP_MAX_STREAMS 1024        /* generator streams of one draw                       */
#define MPPI_NP_MAX_NORMALS 2147483647LL

/* NumPy's RandomState.get_state()[1:5]: the MT19937 key array, its position,
 * and the cached Gaussian of legacy_gauss. */
typedef struct {
    unsigned key[624];
    int pos;
    int has_gauss;
    double gauss;
} mppi_np_state;

/* Where the draw goes: the standard normals z of shape (K, T, du) (C order,
 * n = K T du of them) become out(t, k, d) = (float)(x + mean[d]) with
 *   dot2 = 0: x = z[k][t][src[d]] * scale[d] (NumPy's np.dot when its matrix
 *             has one nonzero per column: the other products are exact zeros),
 *   dot2 = 1 (du = 2, any matrix): x = fma(z[k][t][1], mat[2 + d],
 *             z[k][t][0] * mat[d]) — np.dot(z, mat) as the host BLAS rounds a
 *             2-term product (pinned on the host at run time, hostrng.dot2_model),
 * (fp64, each operation rounded as NumPy's, `x += mean`; then the fp32
 * rounding of the upload), stored at
 * out_dev[t * stride_t + (k - k_offset) * stride_k + d * stride_d]
 * for the samples k_offset <= k < k_offset + K_local of this rank (every rank
 * draws the whole stream, as every rank of the reference's loop would). */
typedef struct {
    void *out_dev;
    long long K, T;
    int du;
    long long k_offset, K_local;
    long long stride_t, stride_k, stride_d;
    int src[MPPI_NP_MAX_DU];
    double scale[MPPI_NP_MAX_DU];
    double mean[MPPI_NP_MAX_DU];
    int dot2;                 /* 1: the general 2 x 2 transform mat (row-major, z @ mat) */
    double mat[4];
} mppi_np_target;

typedef struct mppi_np_ctx mppi_np_ctx;

/* log_params: MPPI_NP_LOG_DATA doubles (mppi_np_log_params). */
int mppi_np_ctx_create(int device, const double *log_params, mppi_np_ctx **out);
void mppi_np_ctx_destroy(mppi_np_ctx *ctx);
/* The generator partition of a draw of n normals from a state at position
 * pos: *streams streams of *block_stride key arrays; stream s >= 1 starts from
 * the jump polynomial x^(624 (block_stride s - 1)) mod P. */
int mppi_np_plan(const mppi_np_ctx *ctx, long long n, int pos, int has_gauss, int *block_stride, int *streams);
/* Upload the polynomials of streams 1 .. streams - 1 (words = MPPI_NP_POLY_WORDS each, row-major). */
int mppi_np_set_jumps(mppi_np_ctx *ctx, int block_stride, int streams, const unsigned long long *polys, int words);
/* Queue the draw of n normals from state *st on `stream` (a hipStream_t) into tgt;
 * asynchronous: mppi_np_draw_result waits for it and returns the state the
 * draw leaves (MPPI_E_RETRY: the output incomplete, the state untouched). */
int mppi_np_draw(mppi_np_ctx *ctx, void *stream, const mppi_np_state *st, long long n, const mppi_np_target *tgt);
int mppi_np_draw_result(mppi_np_ctx *ctx, mppi_np_state *st_out);

#ifdef __cplusplus
}
#endif
#endif /* MPPI_ROCM_H */

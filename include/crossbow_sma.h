/*
 * crossbow_sma.h -- C-ABI of the MI355X-native synchronous model averaging
 * (SMA) path of Crossbow.  Library: crossbow_amd/libcrossbow_sma.so
 * (hipcc, gfx950).  Plain C types only; no HIP or torch types cross it.
 *
 * The entry points are the ones Crossbow's JNI glue binds for the model path
 * (clib-multigpu/GPU.c, header clib-multigpu/uk_ac_imperial_lsds_crossbow_device_TheGPU.h).
 * Each declaration cites the JNI native it replaces.  The reference keeps a
 * process-global context (static theGPU, GPU.c:12); this ABI passes it as an
 * explicit handle and the JNI shim (crossbow_amd/csrc/jni/) keeps the global.
 *
 * Error behaviour: the reference prints and exit(1)s on every failure
 * (clib-multigpu/debug.h:37-57).  Here every function returns a status
 * (CBX_OK or a negative CBX_ERR_*), cbx_last_error() holds the message, and
 * the JNI shim restores "fatal = process exit".  Functions documented as
 * returning a count return it when >= 0.
 */
#ifndef CROSSBOW_SMA_H_
#define CROSSBOW_SMA_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBX_ABI_VERSION 1

#define CBX_OK               0
#define CBX_ERR_INVALID     -1  /* bad argument                                   */
#define CBX_ERR_STATE       -2  /* call out of order (e.g. sync before manager)   */
#define CBX_ERR_HIP         -3  /* HIP runtime failure                            */
#define CBX_ERR_RCCL        -4  /* RCCL failure                                   */
#define CBX_ERR_IO          -5  /* checkpoint file I/O                            */
#define CBX_ERR_NO_DEVICE   -6  /* no usable MI355X (gfx950) device               */
#define CBX_ERR_BARRIER     -7  /* BSP barrier could not lock every replica       */
#define CBX_ERR_UNSUPPORTED -8  /* outside this library's scope   */

/* Update model ids, uk/ac/imperial/lsds/crossbow/types/UpdateModel.java:5 */
#define CBX_UPDATE_DEFAULT           0   /* single GPU: synch/default.c, optimisers/default.cu */
#define CBX_UPDATE_WORKER            1   /* synchronous SGD: synch/synchronoussgd.c */
#define CBX_UPDATE_SYNCHRONOUSEAMSGD 3   /* routed to SMA: clib-multigpu/utils.h:56-57 */
#define CBX_UPDATE_SMA               7

/* Synchronisation models, types/SynchronisationModel.java:5 */
#define CBX_SYNC_BSP 0
#define CBX_SYNC_SSP 1
#define CBX_SYNC_ASP 2

/* Per-model buffers, clib-multigpu/model.h:22-87 */
#define CBX_BUF_DATA     0   /* base: z ; replica: w                    */
#define CBX_BUF_GRADIENT 1   /* base: acc (Phase A output)              */
#define CBX_BUF_DIFF     2   /* base: D (all-reduced) ; replica: s      */
#define CBX_BUF_LAST     3   /* momentum buffer; exists iff momentum>0  */

typedef struct cbx_context cbx_context;

int         cbx_abi_version (void);
const char *cbx_last_error (void);
/* Number of visible gfx950 devices (0 on a host without one). */
int         cbx_device_count (int *count);

/* ---- execution context ------------------------------------------------ */
/* TheGPU.init([I...)  GPU.c:21-63 -> executioncontext.c:152-345.
 * One process drives `ndevices` local GPUs; RCCL comms via ncclCommInitAll
 * (executioncontext.c:185-201), indexed by rank, not device id.          */
int cbx_init (cbx_context **ctx, const int *devices, int ndevices);
/* One process per GPU (torch.distributed launch): rank r of n drives one
 * device; `unique_id` (128 bytes) comes from cbx_get_unique_id on rank 0. */
int cbx_get_unique_id (unsigned char unique_id[128]);
int cbx_init_rank (cbx_context **ctx, int device, int nranks, int rank,
		const unsigned char unique_id[128]);
/* TheGPU.free()  GPU.c:65-75 -> executioncontext.c:728-898 */
int cbx_free (cbx_context *ctx);

/* ---- model registration (Model.GPURegister, Model.java:338-371) ------- */
/* TheGPU.setModel(II)                      GPU.c:672-681  */
int cbx_set_model (cbx_context *ctx, int variables, int bytes);
/* TheGPU.setModelVariable(II[II)           GPU.c:683-696  */
int cbx_set_model_variable (cbx_context *ctx, int id, int order, int ndims,
		const int *shape, int capacity);
/* TheGPU.setModelVariableBuffer(IILjava/nio/ByteBuffer;)  GPU.c:698-708 */
int cbx_set_model_variable_buffer (cbx_context *ctx, int id, int order, const void *src);
/* TheGPU.setModelVariableLearningRateMultiplier(IIF)  GPU.c:710-719.  Stored
 * (executioncontext.c:1592-1605); the SMA optimiser step ignores it, as the
 * reference's does (optimisers/sma.cu uses the solver rate only).         */
int cbx_set_model_variable_learning_rate_multiplier (cbx_context *ctx, int id, int order, float multiplier);
/* TheGPU.setModelWorkPerClock(I)           GPU.c:721-730  */
int cbx_set_model_work_per_clock (cbx_context *ctx, int wpc);
/* TheGPU.setUpdateModelType(I)             GPU.c:732-741; 3 and 7 accepted */
int cbx_set_update_model_type (cbx_context *ctx, int type);

/* ---- solver (SolverConf.GPURegister, SolverConf.java:355-409) --------- */
/* TheGPU.setLearningRateDecayPolicy*  GPU.c:743-821 */
int cbx_set_learning_rate_decay_policy_fixed (cbx_context *ctx, float rate);
int cbx_set_learning_rate_decay_policy_inv (cbx_context *ctx, float rate, double gamma, double power);
int cbx_set_learning_rate_decay_policy_step (cbx_context *ctx, float rate, double gamma, int size);
int cbx_set_learning_rate_decay_policy_multistep (cbx_context *ctx, float rate, double gamma,
		int warmuptasks, int nsteps, const int *steps);
int cbx_set_learning_rate_decay_policy_exp (cbx_context *ctx, float rate, double gamma);
/* TheGPU.setLearningRateDecayPolicyCircular([FI[FI)  GPU.c:803-822: rate[3],
 * momentum[3]; stored, and a learning-rate query then fails with
 * CBX_ERR_UNSUPPORTED as the reference's does (solverconfiguration.c:155-157). */
int cbx_set_learning_rate_decay_policy_circular (cbx_context *ctx, const float *rate, int superconvergence,
		const float *momentum, int step);
/* TheGPU.setBaseModelMomentum(F)  GPU.c:823-832 (stored, unused: sma.c:152) */
int cbx_set_base_model_momentum (cbx_context *ctx, float momentum);
/* TheGPU.setMomentum(FI)          GPU.c:834-843 */
int cbx_set_momentum (cbx_context *ctx, float momentum, int method);
/* TheGPU.setWeightDecay(F)        GPU.c:845-854 */
int cbx_set_weight_decay (cbx_context *ctx, float decay);
/* TheGPU.setEamsgdAlpha(F)        GPU.c:856-865 */
int cbx_set_eamsgd_alpha (cbx_context *ctx, float alpha);
/* TheGPU.setEamsgdTau(I)          GPU.c:867-876 */
int cbx_set_eamsgd_tau (cbx_context *ctx, int tau);

/* ---- model manager ---------------------------------------------------- */
/* TheGPU.setModelManager(II)  GPU.c:878-886 -> executioncontext.c:1720-1764:
 * finalise, push theModel, one base model per GPU, `replicas` per GPU placed
 * round-robin (replica j*G+d on device d, modelmanager.c:51-64).           */
int cbx_set_model_manager (cbx_context *ctx, int replicas, int type);

/* ---- the barrier path (ModelManager.trySynchronise, ModelManager.java:293-353) */
/* TheGPU.lockAny()   GPU.c:1113-1120 -> executioncontext.c:2197-2211.
 * Returns the locked count (BSP: the replica count, or CBX_ERR_BARRIER).  */
int cbx_lock_any (cbx_context *ctx);
/* TheGPU.merge(Z)    GPU.c:1122-1131 -> executioncontext.c:2219-2245.
 * *first = first locked replica id, or -1 when no locked replica has an
 * update (the JNI return value).                                          */
int cbx_merge (cbx_context *ctx, int pull, int *first);
/* TheGPU.synchronise(IIIZ)  GPU.c:1133-1140 -> executioncontext.c:2262-2334
 * -> synch/sma.c:233-248.  Enqueues the SMA step on each device's model
 * synchronisation stream and returns without blocking the host.  Update
 * models SMA (7) and SYNCHRONOUSEAMSGD (3) run SMA; WORKER (1) runs the
 * synchronous-SGD barrier (synch/synchronoussgd.c:13-106, needs the work
 * per clock); DEFAULT (0) copies the base model to every locked replica
 * (synch/default.c:5-43; one GPU only, as in the reference: more devices
 * give CBX_ERR_UNSUPPORTED); any other is CBX_ERR_UNSUPPORTED.          */
int cbx_synchronise (cbx_context *ctx, int first, int clock, int autotune, int push);
/* The same step for a model manager whose buffers live in host memory
 * (north_star: "starts and ends in host memory", databuffer.c:95-122):
 * result-identical to cbx_stage_in + cbx_synchronise + cbx_stage_out, but
 * the flat buffers are cut into `buckets` (1..4096) and the pinned H2D of
 * bucket k+1 and the D2H of bucket k-1 run beside the kernels of bucket k
 * on their own streams, so the step costs about max(H2D, D2H) of PCIe time
 * instead of the sum.  Async like cbx_synchronise; cbx_wait / the step
 * event cover the downloads.  The reference has no such call (its `push`
 * argument is unused, executioncontext.c:2264); update model WORKER runs
 * the three calls unpipelined.                                            */
int cbx_synchronise_staged (cbx_context *ctx, int first, int clock, int autotune, int buckets);
/* TheGPU.unlockAny() GPU.c:1142-1149 -> modelmanager.c:233-245           */
int cbx_unlock_any (cbx_context *ctx);

/* ---- checkpoint / resume ---------------------------------------------- */
/* TheGPU.checkpointModel(String)   GPU.c:1151-1163 -> executioncontext.c:2340-2367.
 * Waits as cbx_wait does, so it refuses (CBX_ERR_STATE) to store a model a
 * poisoned peer-read step left undefined (cbx_peer_import below). */
int cbx_checkpoint_model (cbx_context *ctx, const char *dir);
/* TheGPU.overrideModelData(String) GPU.c:1165-1176 -> executioncontext.c:2369-2388.
 * Drains the streams without that check: loading a checkpoint is a way back. */
int cbx_override_model_data (cbx_context *ctx, const char *dir);
/* Batch-norm running statistics in the checkpoint.  After the model files,
 * executioncontext.c:2352-2364 / 2375-2386 walk the dataflow's BATCHNORM
 * operators and call crossbowCudnnBatchNormParams{Store,Load}Estimated-
 * MeanAndVariable (cudnn/cudnnbatchnormparams.c:102-143) with the
 * operator's id.  The dataflow stays with the caller, so it registers each
 * BN operator's buffers here once (where executioncontext.c:1280-1290 sets
 * them per device); cbx_checkpoint_model / cbx_override_model_data then
 * store / load gpu-%02d-bn-avg-%03d.dat and gpu-%02d-bn-var-%03d.dat
 * (global device id, op id; raw fp32, `elements` floats) in the same
 * directory as the model files.  mean/variance[k]: device pointers on
 * LOCAL device k; a device whose pair is both NULL holds no copy and is
 * skipped (:110-111).  Registering an op again replaces it; elements == 0
 * removes it.                                                             */
int cbx_register_batchnorm_stats (cbx_context *ctx, int op, int elements,
		float *const *mean, float *const *variance);
/* TheGPU.addModel() / delModel()   GPU.c:1178-1199 (autotune; also called
 * by cbx_synchronise for autotune > 0 / < 0, executioncontext.c:2321-2328).
 * add: one new replica per device, ids size .. size+G-1 (id size+g on device
 * g), each a copy of device g's first replica (all four buffers and its
 * solver state, modelmanager.c:362-470, model.c:202-306), left locked for the
 * barrier's unlockAny.  New buffers get their own allocation: pointers
 * returned earlier stay valid.  del: drops ids size-G .. size-1
 * (modelmanager.c:473-557); CBX_ERR_STATE if that would leave none.      */
int cbx_add_model (cbx_context *ctx);
int cbx_del_model (cbx_context *ctx);

/* ---- batch-norm running statistics ----------------------------------- */
/* crossbowCudnnBatchNormParamsSynchroniseEstimatedMeanAndVariable
 * (cudnn/cudnnbatchnormparams.c:157-222; its caller is commented out at
 * executioncontext.c:2268, so this is opt-in), for `layers` BN layers in
 * one all-reduce.  mean/variance[k * layers + l] are device pointers of
 * layer l (elements[l] floats) on LOCAL device k; updated[k * layers + l]
 * is that layer's "updates > 0" on that device.  Per layer, the default
 * device (global device 0) always counts and every other device counts iff
 * updated; every device ends with (sum of counted) / count (unscaled when
 * count == 1).  No-op with one device (:165-166).  Device-synchronises
 * before and after, as the reference does (:171, :218).  The sum order is
 * RCCL's, not device order: equal to the reference within fp32 rounding. */
int cbx_average_batchnorm_stats (cbx_context *ctx, int layers, const int *elements,
		float *const *mean, float *const *variance, const int *updated);

/* ---- task-side replica access (modelmanager.c:147-204) ---------------- */
int cbx_replica_lock (cbx_context *ctx, int id);       /* crossbowModelManagerGet   */
int cbx_replica_unlock (cbx_context *ctx, int id);     /* crossbowModelManagerRelease */
int cbx_replica_task_done (cbx_context *ctx, int id);  /* callbackhandler.c:149-165: updates++ */
int cbx_replica_clock (cbx_context *ctx, int id);
/* crossbowSolverConfGetLearningRate (solverconfiguration.c:116-162) on the
 * replica's own configuration: may raise its _copy flag (LR drop).        */
int cbx_replica_learning_rate (cbx_context *ctx, int id, int task, float *rate);
int cbx_replica_get_copy (cbx_context *ctx, int id);
int cbx_replica_set_copy (cbx_context *ctx, int id, int flag);
/* ---- the theta queue: which replica a task runs on -------------------- */
/* The model manager's theta queue (thetaqueue.c, modelmanager.c:121-132)
 * has one slot per replica id: free, reserved by a task, or disabled.
 * TheGPU.acquireAccess([I)  GPU.c:888-903 -> modelmanager.c:180-190:
 * reserve the next enabled replica of this process in round-robin order,
 * waiting (spinning) until it is free; returns its id and sets *clock to
 * its clock.  CBX_ERR_STATE if every replica here is disabled (the
 * reference spins forever).                                              */
int cbx_acquire_access (cbx_context *ctx, int *clock);
/* TheGPU.upgradeAccess(Integer,[I)  GPU.c:905-921 -> modelmanager.c:192-198:
 * refresh *clock of a reserved replica and return 1, or return 0 (Java
 * null: the task processor re-acquires) once that replica is gone.       */
int cbx_upgrade_access (cbx_context *ctx, int id, int *clock);
/* crossbowModelManagerGetNextOrWait (modelmanager.c:147-167), the execute
 * paths that pick the replica natively (executioncontext.c:2018, 2130):
 * reserve the next replica, wait until its clock >= bound, lock it.
 * Returns its id.  Blocks until a barrier advances the clock.            */
int cbx_get_next_or_wait (cbx_context *ctx, int bound);
/* crossbowModelManagerRelease (modelmanager.c:200-204), from the callback
 * handler after a task (callbackhandler.c:155): unlock the replica and free
 * its theta slot.  CBX_ERR_STATE if the slot is not reserved.             */
int cbx_replica_release (cbx_context *ctx, int id);
/* Disable (flag 1) or re-enable (0) a replica's theta slot
 * (crossbowThetaQueueDisable / Enable, thetaqueue.c:182-206; delModel
 * disables the slots of the replicas it removes).  lockAny then counts it,
 * so BSP still holds, but does not lock it, so the step, unlockAny and the
 * clock leave it alone (modelmanager.c:217-222).  Disabling returns 0, or 1
 * when a task holds the reservation (the slot stays enabled, :199-201);
 * enabling a reserved slot is CBX_ERR_STATE (:182-184).                   */
int cbx_replica_set_disabled (cbx_context *ctx, int id, int flag);
/* crossbowKernelOptimiserSMA (kernels/optimisers/sma.cu:3-100), fused into
 * one pass: the replica's local step for task `task`, which produces the
 * snapshot s (replica->diff) and the new w that the next synchronise()
 * averages.  The learning rate comes from the replica's solver
 * configuration (may raise its _copy flag, solverconfiguration.c:133,147).
 * Enqueued on `stream` (a hipStream_t; NULL = the replica device's sync
 * stream); the sync stream waits for it (sma.cu:79-81) from the library's
 * next call that works on the device (synchronise, wait, staging, reads,
 * writes, add / del, free): the wait is queued then, not at once, so it is
 * not pending on another hardware queue while the update runs.
 * The library keeps one event per caller stream with an update whose wait
 * it has not yet seen complete: a stream it has not seen first drops the
 * entries whose event has completed (their update is done), so task
 * streams that come and go leave nothing behind; at 64 entries per device
 * the pending waits are queued on the sync stream at once (and, if that
 * frees none, the oldest entry's event is waited for on the host).
 * cbx_task_wait_count reports the table's size.  Nesterov
 * momentum is CBX_ERR_UNSUPPORTED, as in the reference (sma.cu:46-48).
 * Under update model WORKER the step is crossbowKernelOptimiserSynchronousSGD
 * (synchronoussgd.cu:3-56) instead: weight decay, then the lr-scaled
 * gradient is added into the device's base-model gradient on the sync
 * stream, to be all-reduced and applied at the next barrier.  Under
 * DEFAULT it is crossbowKernelOptimiserDefault (default.cu:3-131): the
 * replica and its device's base model take the same step, in one pass on
 * the sync stream (the task stream waits for it).                       */
int cbx_replica_optimise (cbx_context *ctx, int id, int task, void *stream);
/* Entries in local device `local`'s table of deferred task-stream waits
 * (see cbx_replica_optimise; at most 64). */
int cbx_task_wait_count (cbx_context *ctx, int local);
/* Global device index a replica lives on (id % G). */
int cbx_replica_device (cbx_context *ctx, int id);
/* 1 if the replica lives in this process. */
int cbx_replica_is_local (cbx_context *ctx, int id);

int cbx_num_replicas (cbx_context *ctx);       /* R * G (modelmanager->size) */
int cbx_num_devices (cbx_context *ctx);        /* G, all ranks               */
int cbx_num_local_devices (cbx_context *ctx);
int cbx_local_device_index (cbx_context *ctx, int local); /* global index    */
long long cbx_model_elements (cbx_context *ctx);

/* ---- buffers ---------------------------------------------------------- */
/* Device pointers (for the task-side kernels that produce w and s).       */
int cbx_replica_buffer (cbx_context *ctx, int id, int kind, void **dev_ptr);
int cbx_base_buffer (cbx_context *ctx, int device, int kind, void **dev_ptr);
/* Blocking copies of a whole buffer (model->bytes) to/from host memory.   */
int cbx_replica_write (cbx_context *ctx, int id, int kind, const void *src, size_t bytes);
int cbx_replica_read (cbx_context *ctx, int id, int kind, void *dst, size_t bytes);
int cbx_base_write (cbx_context *ctx, int device, int kind, const void *src, size_t bytes);
int cbx_base_read (cbx_context *ctx, int device, int kind, void *dst, size_t bytes);

/* Pinned-host staging of the synchronisation buffers (databuffer.c:95-122).
 * stage_in pushes z, last, s_i, w_i; stage_out pulls z, last, w_i.  Async on
 * the sync stream(s); host views are the pinned mirrors below.            */
int cbx_stage_in (cbx_context *ctx);
int cbx_stage_out (cbx_context *ctx);
int cbx_replica_host_buffer (cbx_context *ctx, int id, int kind, void **host_ptr);
int cbx_base_host_buffer (cbx_context *ctx, int device, int kind, void **host_ptr);
/* Block until every local sync stream has drained.  One process per GPU
 * with the peer-read form imported: CBX_ERR_STATE if a drained step on this
 * rank may have read a failed rank's buffers (its poison check found a
 * broken word, cbx_peer_import below): this rank's z and last are then
 * undefined, until cbx_resync_base. */
int cbx_wait (cbx_context *ctx);
/* The event (a hipEvent_t, as void*) recorded on local device `local`'s sync
 * stream at the end of every synchronise(): it stands for the reference's
 * base->updated, synched[dev] and each locked replica's replica->updated
 * (sma.c:115,177,204,222), which this pipeline completes at the same point.
 * Task-side streams wait on it before using a replica again.  Query it
 * after each synchronise(): with timing on it is the stop event the step's
 * last dispatch timestamps (no extra marker), so the handle changes.      */
int cbx_step_event (cbx_context *ctx, int local, void **event);

/* ---- measurement ------------------------------------------------------ */
#define CBX_T_KERNEL    0   /* fused kernel, or kernel A (G > 1)       */
#define CBX_T_ALLREDUCE 1   /* RCCL all-reduce (G > 1)                 */
#define CBX_T_APPLY     2   /* kernel B (G > 1)                        */
#define CBX_T_STEP      3   /* whole synchronise() on the device (staged: incl. copies) */
#define CBX_T_H2D       4   /* last cbx_stage_in, or uploads of the last staged step   */
#define CBX_T_D2H       5   /* last cbx_stage_out, or downloads of the last staged step */
#define CBX_T_COUNT     6
/* When enabled, HIP events bracket each launch on the sync stream.       */
int cbx_set_timing (cbx_context *ctx, int enable);
/* Stream-order check, a debug aid (event-ordering assertions).
 * When on (it turns timing on too), every split step -- kernel A /
 * collective / kernel B per bucket, G > 1 or forced -- records per-bucket
 * timestamps of its last two steps.  cbx_check_order then blocks on them
 * and verifies, per device, that each bucket's collective started after
 * its kernel A ended, that kernel B started after its collective and after
 * the previous B, and that the later step's kernel A(k) started after the
 * earlier step's B(k) (or its last B, when the later step joined the whole
 * stream).  Returns the number of steps checked (0..2 per device), or
 * CBX_ERR_STATE naming the first violation.  Checked steps are consumed; to
 * check cross-step overlap, run two steps back to back between checks.
 * The peer-read and host-staged steps are not recorded.                   */
int cbx_set_order_check (cbx_context *ctx, int enable);
int cbx_check_order (cbx_context *ctx);
/* Milliseconds of the last step on local device `local`, CBX_T_COUNT floats
 * (blocks on the recorded events); -1 for a span the step did not have.   */
int cbx_last_timing (cbx_context *ctx, int local, float *ms);
/* Per-launch history of the last steps (up to 1024) on local device `local`:
 * `which` is CBX_T_KERNEL, CBX_T_ALLREDUCE, CBX_T_APPLY or CBX_T_STEP; fills
 * ms[0..count) oldest first and returns count.  For a pipelined split step
 * (2..64 buckets, order check off; the last 64 such steps) KERNEL, ALLREDUCE
 * and APPLY are the step's summed busy spans of kernels A, collectives and
 * kernels B: each dispatch's stop minus the latest event that bounded its
 * start (the previous dispatch on its stream, the events the stream waited
 * on), so each includes its dispatch latency and any sharing of the GPU
 * with the other streams' work.  Both this and cbx_last_timing report -1
 * for a span a step did not keep.                                         */
int cbx_timing_history (cbx_context *ctx, int local, int which, float *ms, int max);
/* Launch geometry for the SMA kernels: threads per block (multiple of 64),
 * workgroups per CU for the grid-stride loop (0 = one float4 per thread),
 * load/store policy (0 plain, 1 nontemporal), float4s per thread per trip. */
int cbx_set_kernel_config (cbx_context *ctx, int block, int blocks_per_cu, int policy, int unroll);
/* Occupancy cap for the SMA kernels, in waves per CU: 1..32, 0 = none, -1
 * = auto (the default: about 56 buffer streams, reads plus writes, in
 * flight per CU, i.e. 2 waves for the R = 8 step, 11 for kernel B, 8 for
 * the optimiser step).  Enforced through reserved LDS per
 * workgroup (so the smallest reachable cap is 2 workgroups per CU).      */
int cbx_set_kernel_occupancy (cbx_context *ctx, int waves_per_cu);
/* Launch geometry of the per-task kernels (the replica optimiser step and
 * the S-SGD task/barrier kernels): threads per block (64..512, multiple of
 * 64), float4s per lane (1 or 2), occupancy cap in waves per CU as above. */
int cbx_set_aux_kernel_config (cbx_context *ctx, int block, int unroll, int waves_per_cu);
/* Launch geometry of the write-heavy barrier kernels (the DEFAULT broadcast
 * and the S-SGD apply), same arguments as above; defaults are per kernel
 * (256 / 1 / 8 and 64 / 2 / 3, measured).                                */
int cbx_set_barrier_kernel_config (cbx_context *ctx, int block, int unroll, int waves_per_cu);
/* Launch geometry of kernel B of the G > 1 split SMA path (Phase C,
 * sma.c:135-183: 3 reads + 2 writes per element): block 64..256, unroll 1,
 * 2 or 4, occupancy cap as above.  Default 64 / 2 / auto.                 */
int cbx_set_apply_kernel_config (cbx_context *ctx, int block, int unroll, int waves_per_cu);
/* Bucketed pipeline for G > 1: kernel A / all-reduce / kernel B per bucket
 * of `bucket_elements` floats; 0 (default) = 8 buckets when G > 1, one at
 * G = 1; a value >= n = one bucket, all in order on the sync stream.  With
 * more than one bucket the all-reduce of bucket k runs on a second stream
 * beside kernel A of bucket k+1, and the kernels are timed as summed busy
 * spans (cbx_timing_history).                                             */
int cbx_set_bucket_elements (cbx_context *ctx, long long bucket_elements);
/* How the bucketed pipeline overlaps (G > 1, or forced split): 0 (default)
 * within a step only; 1 also across steps: kernels A run on their own
 * stream and A(k) waits only for B(k) of the previous step, so the next
 * step's first buckets run while this step's last all-reduces are on the
 * link.  Any other C-ABI call between two steps that may enqueue device
 * work makes the next step join the whole sync stream first.  Same results
 * bit for bit in both modes.                                              */
int cbx_set_pipeline_mode (cbx_context *ctx, int mode);
/* Mode 1: kernel A(k) waits for kernel B of the previous step once
 * per `stride` buckets, on B(k + stride - 1), which implies the earlier
 * ones.  1 (default) waits per bucket; larger strides pay fewer
 * cross-queue waits for less overlap between steps.  1..4096.            */
int cbx_set_cross_wait_stride (cbx_context *ctx, int stride);
/* Split path with buckets (every pipeline mode): all-reduce `group`
 * buckets behind one wait of the all-reduce stream on kernel A of the
 * group's last bucket, instead of one wait per bucket.  1 (default) is the
 * per-bucket order.  Larger groups pay fewer cross-queue waits (~10 us of
 * queue latency each) and start each group's all-reduces later.  Same
 * results bit for bit.  1..4096.  No reference counterpart: the bucket
 * pipeline itself is this library's (common.c:14-54 all-reduces one flat
 * buffer).                                                                */
int cbx_set_allreduce_group (cbx_context *ctx, int group);
/* How the SMA step's all-reduce crosses devices (G > 1):
 *   CBX_ALLREDUCE_RCCL (0, default): grouped ncclAllReduce, bucketed and
 *     pipelined as configured above (synch/common.c:3-57);
 *   CBX_ALLREDUCE_PEER (1): one process over every device (cbx_init with G
 *     devices), or one process per GPU once cbx_peer_import has mapped every
 *     rank's buffers (below).  No RCCL pass: after hipDeviceEnablePeerAccess
 *     (or the IPC mapping), device g sums shard g of every device's acc by
 *     direct peer reads, then
 *     kernel B on each device reads every shard of D from its owner
 *     (two-shot over all xGMI links at once; the reference's non-NCCL path
 *     copies peer buffers, common.c:64-95).  Bucketed and pipelined like
 *     the all-reduce (bucket size, modes, strides, groups above): the
 *     reduction of bucket k runs on the all-reduce stream beside kernel A of
 *     bucket k+1 and waits for kernel A(k) of EVERY device; kernel B(k) waits
 *     for every device's reduction of k.  Sums in device order: bit-exact
 *     against the rank-order oracle and identical on every device.  The
 *     host-staged step and S-SGD keep RCCL.
 *   CBX_ALLREDUCE_RSAG (2): every process form.  Per bucket, RCCL
 *     reduce-scatter of acc (the control block rides a grouped 64-float
 *     all-reduce), the base momentum on this rank's shard only
 *     (last = fma(0.9, last, D)), RCCL all-gather of last, then kernel B
 *     adds the gathered D' to z.  The all-reduce's link bytes; the momentum
 *     pass (12 B per element) runs on 1/G of the bucket; every rank ends
 *     with the same z and last (SURVEY 8(e) variant 1).  G must divide 1024
 *     (powers of two up to 16).  The host-staged step and S-SGD keep the
 *     all-reduce.
 * CBX_ERR_STATE for PEER on a one-process-per-GPU context before
 * cbx_peer_import.                                                         */
#define CBX_ALLREDUCE_RCCL 0
#define CBX_ALLREDUCE_PEER 1
#define CBX_ALLREDUCE_RSAG 2
int cbx_set_allreduce_algorithm (cbx_context *ctx, int algorithm);
/* The peer-read all-reduce with one process per GPU (cbx_init_rank, G > 1;
 * no reference counterpart: the reference runs one process over every GPU,
 * executioncontext.c:185-201, and its non-NCCL path copies peer buffers,
 * common.c:64-95).  After cbx_set_model_manager on every rank:
 *   1. cbx_peer_export(ctx, blob, &bytes) writes this rank's handles into
 *      `blob` (CBX_PEER_BLOB_BYTES): the IPC handles (hipIpcGetMemHandle)
 *      of its acc and D buffers, which move out of the model arena into
 *      allocations of their own (below 2 GiB - 2 MiB each: ROCm 7.0's IPC
 *      keeps an allocation's size in 32 bits, and an open of 2 GiB or more
 *      never returns; CBX_ERR_UNSUPPORTED above); rank 0
 *      also creates the page of completion flags (POSIX shared memory) and
 *      names it in its blob;
 *   2. the caller gathers every rank's blob, in rank order, over its own
 *      control plane (bench.py: gloo all_gather);
 *   3. cbx_peer_import(ctx, blobs, nranks) maps every other rank's acc and
 *      D (hipIpcOpenMemHandle; the ranks open in turn; a rank that has not
 *      opened its handles 120 s into the import fails everyone's import) and
 *      pins the flag page
 *      (hipHostRegister).  It succeeds on every rank or on none: a rank
 *      whose opens failed fails every rank's import.
 * Then CBX_ALLREDUCE_PEER is accepted.  The ranks' streams order each
 * other through the flags: a rank writes the step's sequence number after
 * its kernel A / reduction of a bucket (hipStreamWriteValue64), the others
 * wait for it (hipStreamWaitValue64 >=); the pipeline, its modes, strides,
 * groups and the sums' device order are the single-process form's.  Same
 * results bit for bit.  At most 4096 buckets.  cbx_free then waits (up to
 * 60 s in all, streams polled) until every rank is done with this rank's
 * memory; if a dead peer left this rank's streams waiting, it writes the
 * release into every rank's flags itself.  Every rank calls export, import
 * and free.
 * Failure (the reference's answer to any failure is exit(1), debug.h:37; the
 * invariant at stake is that every GPU applies the same D to the same z,
 * synch/sma.c:168-174):
 *   - A step that fails part-way on a rank (its call returns the error; that
 *     rank's z, last and replicas are undefined from it on, as for a
 *     poisoned step) sets that rank's broken word on the page, then releases
 *     its flags (from the host, and again behind its queued flag writes), so
 *     no other rank's stream waits forever.
 *   - A released flag lets a wait pass whether or not the data it guards was
 *     written, so a step another rank had already enqueued may read the
 *     failed rank's stale acc or D.  So after each step's last kernel B, on
 *     the same stream (every load of the step's kernels B has returned), one
 *     wave reads every rank's broken word and, if one is set, records the
 *     step's sequence number on the page.  cbx_wait on that rank then
 *     returns CBX_ERR_STATE naming the
 *     step: its z and last are undefined from that step on.  A step whose
 *     cbx_wait reports nothing read only data that was complete (any stale
 *     read needs a release, and the broken word comes before it).
 *   - From the moment any rank's broken word is visible to a rank, that
 *     rank refuses EVERY collective step (cbx_synchronise and
 *     cbx_synchronise_staged in every all-reduce form and update model, and
 *     cbx_average_batchnorm_stats) with CBX_ERR_STATE, releasing its own
 *     flags first, until cbx_resync_base.  The decision is each rank's own,
 *     made from the page when it is called.  A job that keeps the peer-read
 *     form across steps always recovers (every later step is refused or
 *     reported).  A job that switches to an RCCL collective while a failure
 *     is still on its way to some rank can leave that rank inside a
 *     collective the others refuse; every rank's cbx_resync_base then fails
 *     within its 60 s bounds and the job must end, as the reference's does.
 *     After a failure on any rank, every rank stops stepping and calls
 *     cbx_resync_base.
 * Same results bit for bit as before whenever no rank fails.              */
#define CBX_PEER_BLOB_BYTES 256
int cbx_peer_export (cbx_context *ctx, void *blob, size_t *bytes);
int cbx_peer_import (cbx_context *ctx, const void *blobs, int nranks);
/* Re-synchronise the base models after a failure (or at any time): every
 * rank calls it (a collective over the RCCL communicator).  Releases this
 * rank's flags if it knows of a failure, waits (up to 60 s, polled) until its
 * streams drain, broadcasts z and last (device buffers, padded length) from
 * rank `root`, and, once every rank has drained and received them, clears
 * this rank's flag words, broken and poison words and restarts the form's
 * step numbering; a second barrier keeps every rank from starting a step
 * before every rank's words are clear.  Afterwards z and last are identical
 * on every rank and every form is accepted again.  Replicas (w_i, s_i) are
 * left as they are (a Phase-D copy request resets them to z).  No-op at
 * G = 1.                                                                  */
int cbx_resync_base (cbx_context *ctx, int root);
/* How cbx_synchronise_staged moves the model between the pinned host mirror
 * and the device (north_star: the path starts and ends in host memory):
 *   CBX_STAGING_ZEROCOPY (0, default): the SMA kernels read their inputs
 *     from the host mirror over PCIe and write their outputs to it and to
 *     the device, both link directions at once, no copy engine;
 *   CBX_STAGING_DMA (1): copy-engine uploads and downloads per bucket on
 *     their own streams, overlapping the kernels (databuffer.c:95-122 is the
 *     reference's synchronous staging).
 * Both leave host and device exactly as cbx_stage_in + cbx_synchronise +
 * cbx_stage_out do.                                                        */
#define CBX_STAGING_ZEROCOPY 0
#define CBX_STAGING_DMA 1
int cbx_set_staging_mode (cbx_context *ctx, int mode);
/* One process over several local devices (cbx_init): who enqueues each
 * device's share of a barrier step (the SMA split and peer-read steps).
 *   0   one thread, every device in turn, collectives grouped across the
 *       devices (the reference's ResultCollector thread, common.c:14-54);
 *   1   one thread per local device, each issuing its own device's kernels
 *       and collectives (NCCL's thread-per-device use of ncclCommInitAll's
 *       communicators); the call returns once every device's work is
 *       enqueued, as before;
 *  -1   (default) 0: the reference's form, until measured otherwise on
 *       distinct devices (bench.py's warm-up tuner times 0 against 1).
 * Same work on the same streams in the same per-device order: results are
 * identical (a threaded peer-read step orders its cross-device waits behind
 * the other devices' event records).  At 8 devices and 8 buckets one thread
 * may spend longer enqueuing a step than the GPUs spend running it
 * (DESIGN.md section 6).                                                   */
int cbx_set_enqueue_threads (cbx_context *ctx, int mode);
/* Force the multi-GPU pipeline (kernel A + RCCL all-reduce + kernel B) even
 * at G = 1 (a one-rank communicator), so a single-GPU host exercises it.  */
int cbx_set_force_split (cbx_context *ctx, int force);
/* Synthetic inputs of BASELINE.md 2.3, generated on the device:
 * z ~ N(0,.05^2), s_i = z + N(0,.01^2), w_i = s_i + N(0,.001^2),
 * last ~ N(0,.001^2); seeds derive from `seed` ^ buffer id.               */
int cbx_fill_synthetic (cbx_context *ctx, unsigned long long seed);
/* Float4 device-to-device copy ceiling on local device 0: `bytes` per
 * buffer, `iters` timed launches; writes achieved GB/s (read + write).    */
int cbx_bench_copy (cbx_context *ctx, size_t bytes, int iters, float *gbps);

/* ---- the sma.c seam: buffers owned by the caller ------------------------
 * For a Crossbow build that keeps its own model manager, model buffers and
 * task side (modelmanager.c, model.c, executioncontext.c, the callback and
 * task handlers, all untouched) and replaces only two function bodies:
 *   crossbowSynchronisationSMA (synch/sma.c:233-248 -> :13-231)
 *       -> cbx_sma_plan_step
 *   crossbowKernelOptimiserSMA (kernels/optimisers/sma.cu:3-100)
 *       -> cbx_sma_optimise_buffers
 * (INTEGRATION.md section 3 shows both bodies).  Buffers hold exactly
 * `elements` floats (no padding) and must be 16-byte aligned, as hipMalloc's
 * are.  Same kernels and arithmetic as the context path: bit-exact against
 * the oracle at one GPU and in rank order.  No context is involved.       */
typedef struct cbx_sma_plan cbx_sma_plan;
/* What the step needs beyond the caller's buffers, per device: the Phase-A
 * accumulator and the all-reduced difference (base->gradient, base->diff in
 * sma.c:66,82) with the control block that carries the Phase-D request
 * count, and the communicators: `comms` = the caller's ncclComm_t per device
 * (ctx->comms of executioncontext.c:185-201, as void*), or NULL to create
 * them with ncclCommInitAll over `devices` (ndevices > 1).  `devices` are
 * HIP device ids; `elements` = model->elements (model.h:35).             */
int cbx_sma_plan_create (cbx_sma_plan **plan, const int *devices, int ndevices, long long elements,
                         void *const *comms);
int cbx_sma_plan_free (cbx_sma_plan *plan);
/* G > 1: cut the step into `buckets` buckets and run the all-reduce of
 * bucket k on a stream of the plan's beside kernel A of bucket k+1 (as the
 * context's pipeline does; the caller's stream still orders the step
 * against its other work).  0 (default) = 8 buckets; 1 = the reference's
 * order, everything on the caller's stream.  Same results bit for bit.    */
int cbx_sma_plan_set_buckets (cbx_sma_plan *plan, int buckets);
/* One SMA step (sma.c:13-231), enqueued on the caller's streams, async:
 *   streams[k]        dev->modelSynchronisationStream of devices[k] (hipStream_t)
 *   z[k], last[k]     baseModels[k]->data->dev / ->last->dev (last may be NULL
 *                     when momentum is 0, model.c:116-120)
 *   nreplicas         modelmanager->size; for replica id:
 *     replica_device[id]  position in `devices` of replicas[id]->dev
 *     w[id], s[id]        replicas[id]->data->dev, replicas[id]->diff->dev
 *     locked[id]          modelmanager->locked[id]
 *     copy[id]            replicas[id]->conf->_copy
 *   alpha             defaultModel->conf->alpha (sma.c:33)
 *   momentum          the base model's conf->momentum: > 0 applies the
 *                     hard-coded 0.9 (sma.c:150-152)
 *   first             replicas below it take no part (sma.c:69)
 * Locked replicas at or above `first` are averaged in id order per device.
 * Returns 1 when Phase D ran (a locked replica from `first` on had _copy:
 * every such replica now equals its device's base model; the caller resets
 * their _copy, sma.c:217-220), 0 when not.  The caller's events
 * (base->updated, synched[dev], replica->updated) are recorded on the same
 * streams after the call, as sma.c:115,177,204,222 do.  One step at a time
 * per plan (the reference's single ResultCollector thread): the scratch is
 * the plan's.  streams[k] must be the same stream on every call of a plan
 * (as dev->modelSynchronisationStream is): with buckets, the next step's
 * all-reduce of bucket k is ordered after this step's last kernel B only
 * through that stream, so a different stream would let it overwrite the
 * plan's D while B still reads it.  With a communicator that spans processes, each process
 * passes only its own replicas as locked; a Phase-D request on any rank
 * reaches every rank through the all-reduced control block, so the return
 * value reports this process's requests only.                           */
int cbx_sma_plan_step (cbx_sma_plan *plan, void *const *streams, float *const *z, float *const *last,
                       int nreplicas, const int *replica_device, float *const *w, const float *const *s,
                       const int *locked, const int *copy, float alpha, float momentum, int first);
/* The replica's optimiser step of one task (sma.cu:3-100) in one pass over
 * its buffers, on `stream` (hipStream_t, the task stream; the current HIP
 * device must be the buffers'): w = model->data, g = model->gradient
 * (updated in place, as the reference leaves it), last = model->last (used
 * iff momentum > 0), s = model->diff (the snapshot of w before the update);
 * learning_rate = crossbowSolverConfGetLearningRate (conf, task)
 * (solverconfiguration.c:116-162); momentum, weight_decay from the conf.
 * Nesterov momentum stays the caller's err() (sma.cu:46-48).             */
int cbx_sma_optimise_buffers (void *stream, float *w, float *g, float *last, float *s, long long elements,
                              float learning_rate, float momentum, float weight_decay);
/* The same seam for update model WORKER (synchronous SGD):
 * crossbowSynchronisationSynchronousSGD (synch/synchronoussgd.c:13-106) ->
 * cbx_ssgd_plan_step, over acc[k] = baseModels[k]->gradient->dev (the
 * accumulated lr-scaled task gradients; reset to 0 by the step), z, last
 * (used iff momentum > 0: the base model's conf->momentum, NOT forced to
 * 0.9), the locked replicas from `first` on (set to their device's new base
 * model, common.c:198-220) and wpc = defaultBaseModel->wpc (D *= 1/wpc).
 * Buckets as cbx_sma_plan_set_buckets sets them at G > 1; one rank always
 * runs one apply pass (no all-reduce to overlap), whatever the setting.
 * streams[k] must be the same stream on every call, as for cbx_sma_plan_step.
 * crossbowKernelOptimiserSynchronousSGD (kernels/optimisers/synchronoussgd.cu:
 * 3-56) -> cbx_ssgd_accumulate_buffers: g += weight_decay * w, then
 * acc += -learning_rate * g, on `stream` = the device's model-synchronisation
 * stream once it has waited for the task's gradient (:37-40).            */
/* crossbowCudnnBatchNormParamsSynchroniseEstimatedMeanAndVariable
 * (cudnn/cudnnbatchnormparams.c:157-222) over the caller's statistics
 * buffers: arguments as cbx_average_batchnorm_stats, with k the position in
 * the plan's devices (the default device is rank 0 of the communicator).
 * No-op with one rank.  Device-synchronises before and after.             */
int cbx_sma_plan_average_batchnorm (cbx_sma_plan *plan, int layers, const int *elements, float *const *mean,
                                    float *const *variance, const int *updated);
int cbx_ssgd_plan_step (cbx_sma_plan *plan, void *const *streams, float *const *z, float *const *last,
                        float *const *acc, int nreplicas, const int *replica_device, float *const *w,
                        const int *locked, float momentum, int wpc, int first);
int cbx_ssgd_accumulate_buffers (void *stream, const float *w, float *g, float *acc, long long elements,
                                 float learning_rate, float weight_decay);

#ifdef __cplusplus
}
#endif

#endif /* CROSSBOW_SMA_H_ */

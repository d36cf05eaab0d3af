/*
 * sma_oracle.h -- CPU restatement of Crossbow's synchronous model averaging
 * (SMA) step.  TEST INFRASTRUCTURE ONLY: the checker for the HIP path and the
 * CPU baseline leg of bench.py.  Nothing in crossbow_amd/ may link or call it.
 *
 * Parity status: the reference ships no golden vectors, tests or fixtures for
 * this path and cannot be compiled here (CUDA,
 * cuBLAS, NCCL, JNI).  The restatement is therefore "parity unpinned" with
 * respect to reference-produced outputs.  It IS cross-checked against a real
 * third-party BLAS (OpenBLAS cblas_saxpy, the library the reference links for
 * its CPU path, clib-multigpu/BLAS.c:32,328) replaying the reference's exact
 * call sequence (cbo_sma_blas below): both must agree bit for bit.
 */
#ifndef CROSSBOW_SMA_ORACLE_H_
#define CROSSBOW_SMA_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Hard-coded base-model momentum, clib-multigpu/synch/sma.c:152
 * ("model->conf->momentum = 0.9;" into a float field). */
#define CBO_BASE_MOMENTUM 0.9f

/* ---------------------------------------------------------------------- */
/* Synthetic inputs: splitmix64 -> Box-Muller.   */
/* Counter based: element k of buffer b depends only on (seed ^ b, k).     */
/* ---------------------------------------------------------------------- */
#define CBO_SEED 20190701ULL
enum {
	CBO_BUF_Z = 0,      /* base model data, z            */
	CBO_BUF_LAST = 1,   /* base model momentum, last     */
	CBO_BUF_S0 = 16,    /* replica i snapshot: 16 + 2i   */
	CBO_BUF_W0 = 17     /* replica i data:     17 + 2i   */
};

uint64_t cbo_splitmix64 (uint64_t x);

/* out[k] = (mean ? mean[k] : 0) + sigma * N(0,1)[seed, k]  for k in [0, n) */
void cbo_fill_normal (float *out, size_t n, uint64_t seed, float sigma, const float *mean);

/* ---------------------------------------------------------------------- */
/* The SMA step, multi-GPU semantics (clib-multigpu/synch/sma.c:13-231)    */
/* restated for G "devices" inside one address space.                      */
/*                                                                         */
/*  size       number of replicas (R * G); replica i lives on device i % G */
/*             (round-robin placement, clib-multigpu/modelmanager.c:51-64) */
/*  z[g]       base model data on device g       (base->data)              */
/*  last[g]    base model momentum (NULL iff momentum <= 0, model.c:116)   */
/*  s[i]       replica snapshot                  (replica->diff)           */
/*  w[i]       replica data                      (replica->data)           */
/*  locked[i]  replica participates  (modelmanager.c:206-231)              */
/*  copy[i]    replica conf->_copy flag; reset to 0 when a copy happens    */
/*  first      first replica id considered (sma.c:69)                      */
/*  scratch    G * n floats of workspace (acc per device) + n floats (D)   */
/* Returns the number of replicas whose _copy flag triggered Phase D.      */
/* ---------------------------------------------------------------------- */
int cbo_sma_fma (int G, int size, size_t n, float alpha, float momentum,
		float **z, float **last, float **s, float **w,
		const int *locked, int *copy, int first, float *scratch);

/* Same step, replaying the reference's BLAS call sequence literally:      */
/* memset / memcpy / saxpy(-1) / saxpy(-alpha) / saxpy(+alpha) per replica */
/* (sma.c:66-107), sum over devices (common.c:43-52), saxpy(0.9,last) +    */
/* memcpy (sma.c:155-164), saxpy(1,D,z) (sma.c:169-174), Phase D copies.   */
/* Uses the OpenBLAS loaded by cbo_blas_open.  scratch: 2*G*n + n floats.  */
int cbo_sma_blas (int G, int size, size_t n, float alpha, float momentum,
		float **z, float **last, float **s, float **w,
		const int *locked, int *copy, int first, float *scratch);

/* The two per-device halves of the multi-GPU step, for checking a sharded  */
/* execution (one rank per device) against cbo_sma_fma:                     */
/*  accumulate: Phase A over `R` replicas of ONE device (already filtered   */
/*              to locked ones, id order) -> acc[n]; returns copy requests.  */
/*  apply:      Phase C on the all-reduced D, then Phase D (w_i = z for the */
/*              R listed replicas) when copy != 0.  D is not modified.       */
int cbo_sma_accumulate (int R, size_t n, float alpha, const float *z,
		float **s, float **w, const int *copy, float *acc);
void cbo_sma_apply (int R, size_t n, float momentum, const float *D,
		float *z, float *last, float **w, int copy);

/* The replica's local optimiser step for one task, the producer of s and w */
/* (crossbowKernelOptimiserSMA, clib-multigpu/kernels/optimisers/sma.cu:3-100). */
/* `rate` is the already negated learning rate (sma.cu:43).  `last` may be  */
/* NULL iff momentum <= 0.                                                  */
/*   wd > 0      : g = fma(wd, w, g)                      sma.cu:24-31      */
/*   momentum > 0: g = rate * g; g = fma(mu, last, g);    sma.cu:52-64      */
/*                 last = g; s = w; w = fma(1, g, w)      sma.cu:68-74      */
/*   else        : s = w; w = fma(rate, g, w)             sma.cu:87-90      */
void cbo_sma_optimise (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *s);
/* Same step replaying the reference's cuBLAS/memcpy sequence on OpenBLAS. */
int cbo_sma_optimise_blas (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *s);

/* Synchronous SGD (update model WORKER), the other synchronous model on the  */
/* same buffers.  Task step, crossbowKernelOptimiserSynchronousSGD           */
/* (kernels/optimisers/synchronoussgd.cu:3-56): rate is -learningRate(task). */
/*   g = fma(wd, w, g) if wd > 0 (:20-26);  acc = fma(rate, g, acc) (:46-52)  */
void cbo_ssgd_worker (size_t n, float rate, float wd, const float *w, float *g, float *acc);
int cbo_ssgd_worker_blas (size_t n, float rate, float wd, const float *w, float *g, float *acc);
/* Barrier, synch/synchronoussgd.c:13-106 (+ common.c:3-57, 198-220), G     */
/* devices in one address space.  acc[g] is each device's base gradient.    */
/*   D = sum_g acc_g (rank order); per device: D' = (1/wpc) * D; if         */
/*   momentum > 0: D' = fma(mu, last, D'), last = D'; z = fma(1, D', z);    */
/*   acc_g = 0; every locked replica i >= first on g: w_i = z_g.            */
/* scratch: n floats (blas: 2n).                                            */
void cbo_ssgd_sync (int G, int size, size_t n, int wpc, float momentum,
		float **z, float **last, float **w, float **acc,
		const int *locked, int first, float *scratch);
int cbo_ssgd_sync_blas (int G, int size, size_t n, int wpc, float momentum,
		float **z, float **last, float **w, float **acc,
		const int *locked, int first, float *scratch);

/* DEFAULT update model (0), the reference apps' default (ModelConf.java:81). */
/* Task step, crossbowKernelOptimiserDefault (kernels/optimisers/default.cu: */
/* 3-131): the replica AND its device's base model take the step; rate is   */
/* -learningRate(task).                                                      */
/*   wd > 0      : g = fma(wd, w, g)                          default.cu:26-35   */
/*   momentum > 0: g = rate * g; g = fma(mu, last, g);        default.cu:46-66   */
/*                 last = g; w = fma(1, g, w); z = fma(1, g, z)  :69-99         */
/*   else        : w = fma(rate, g, w); z = fma(rate, g, z)   default.cu:102-127 */
void cbo_default_task (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *z);
int cbo_default_task_blas (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *z);
/* Barrier, single GPU only (synch/default.c:5-43): w_i = z for every locked */
/* replica i >= first.  (Multi-GPU DEFAULT is err() in the reference, :46-51.) */
void cbo_default_sync (int size, size_t n, const float *z, float **w, const int *locked, int first);

/* Batch-norm running-statistics averaging across devices                  */
/* (crossbowCudnnBatchNormParamsSynchroniseEstimatedMeanAndVariable,        */
/* cudnn/cudnnbatchnormparams.c:157-222), for `layers` BN layers at once.   */
/* mean/var[g * layers + l] is layer l's buffer (elements[l] floats) on     */
/* device g; updated[g * layers + l] is that layer's p->updates[g] > 0.     */
/* Per layer: device 0 (the default device) accumulates, in device order,   */
/* M = fma(1, m_g, M) for every other device g with updates (:175-190);     */
/* count = 1 + their number; if count > 1, M *= 1/count (:193-197); every   */
/* other device then receives M (:200-209).  Returns 0.                     */
int cbo_bn_average (int G, int layers, const int *elements, float **mean, float **var, const int *updated);

/* dlopen an OpenBLAS build; returns 0 on success.  `path` may be NULL to  */
/* probe the usual numpy/scipy wheels.  Records the library actually used. */
int cbo_blas_open (const char *path);
const char *cbo_blas_name (void);
void cbo_blas_set_threads (int threads);
int cbo_blas_is_open (void);

/* Bind the calling thread to one core (clib-multigpu/CPU.c:39-52). */
int cbo_bind_core (int core);
int cbo_unbind (void);

/* Wall clock, seconds. */
double cbo_now (void);

#ifdef __cplusplus
}
#endif

#endif /* CROSSBOW_SMA_ORACLE_H_ */

/*
 * sma_oracle.c -- CPU restatement of Crossbow's SMA step.
 *
 * TEST INFRASTRUCTURE ONLY (see sma_oracle.h).  Imported by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg.
 * The product library (crossbow_amd/csrc) never links or calls this file.
 *
 * Every function cites the reference lines it restates.  Arithmetic follows
 * cuBLAS saxpy semantics y := fma(a, x, y) in float32 (one rounding per
 * element), in the reference's operation order.
 */
#define _GNU_SOURCE
#include "sma_oracle.h"

#include <dlfcn.h>
#include <math.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

/* ---------------------------------------------------------------------- */
/* PRNG: splitmix64 (one step from state x) and Box-Muller in double.      */
/* ---------------------------------------------------------------------- */
#define CBO_GOLDEN 0x9E3779B97F4A7C15ULL

uint64_t cbo_splitmix64 (uint64_t x) {
	uint64_t z = x + CBO_GOLDEN;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

static inline double cbo_normal (uint64_t seed, uint64_t k) {
	uint64_t a = cbo_splitmix64 (seed + (2 * k) * CBO_GOLDEN);
	uint64_t b = cbo_splitmix64 (seed + (2 * k + 1) * CBO_GOLDEN);
	double u1 = ((double) ((a >> 11) + 1)) * (1.0 / 9007199254740992.0); /* (0, 1] */
	double u2 = ((double) (b >> 11)) * (1.0 / 9007199254740992.0);       /* [0, 1) */
	return sqrt (-2.0 * log (u1)) * cos (6.283185307179586 * u2);
}

void cbo_fill_normal (float *out, size_t n, uint64_t seed, float sigma, const float *mean) {
	size_t k;
	for (k = 0; k < n; ++k) {
		float v = (float) ((double) sigma * cbo_normal (seed, k));
		out[k] = mean ? (mean[k] + v) : v;
	}
}

/* ---------------------------------------------------------------------- */
/* The SMA step with explicit fmaf (the fast, portable restatement).       */
/* ---------------------------------------------------------------------- */
int cbo_sma_fma (int G, int size, size_t n, float alpha, float momentum,
		float **z, float **last, float **s, float **w,
		const int *locked, int *copy, int first, float *scratch) {

	int g, i, copies = 0;
	size_t k;
	float *acc = scratch;                /* base->gradient per device */
	float *D = scratch + (size_t) G * n; /* reduced base->diff        */

	/* Phase A, clib-multigpu/synch/sma.c:42-128: per device, replicas in
	 * increasing id order, restricted to locked replicas on that device. */
	for (g = 0; g < G; ++g) {
		float *a = acc + (size_t) g * n;
		memset (a, 0, n * sizeof(float));                                   /* sma.c:66 */
		for (i = first; i < size; ++i) {
			if (! locked[i] || (i % G) != g)                                /* sma.c:71 */
				continue;
			for (k = 0; k < n; ++k) {
				float d = fmaf (-1.0f, z[g][k], s[i][k]);                   /* sma.c:79-90 */
				w[i][k] = fmaf (-alpha, d, w[i][k]);                        /* sma.c:93-99 */
				a[k] = fmaf (alpha, d, a[k]);                               /* sma.c:102-107 */
			}
			if (copy[i])                                                    /* sma.c:113-120 */
				copies++;
		}
	}

	/* Phase B, clib-multigpu/synch/common.c:3-57: D = sum_g acc_g.  A
	 * single-rank all-reduce is a copy; otherwise sum in rank order. */
	memcpy (D, acc, n * sizeof(float));
	for (g = 1; g < G; ++g)
		for (k = 0; k < n; ++k)
			D[k] = D[k] + acc[(size_t) g * n + k];

	/* Phase C, sma.c:135-183: base momentum hard-coded to 0.9 when the base
	 * model's momentum is positive; then z += D on every device. */
	for (g = 0; g < G; ++g) {
		for (k = 0; k < n; ++k) {
			float Dg = D[k];
			if (momentum > 0) {
				Dg = fmaf (CBO_BASE_MOMENTUM, last[g][k], Dg);              /* sma.c:155-160 */
				last[g][k] = Dg;                                            /* sma.c:163-164 */
			}
			z[g][k] = fmaf (1.0f, Dg, z[g][k]);                             /* sma.c:169-174 */
		}
	}

	/* Phase D, sma.c:185-227: any locked replica with _copy set makes every
	 * locked replica (on every device) copy its device's base model. */
	if (copies > 0) {
		for (i = first; i < size; ++i) {
			if (! locked[i])
				continue;
			memcpy (w[i], z[i % G], n * sizeof(float));                     /* sma.c:213-217 */
			copy[i] = 0;                                                    /* sma.c:220 */
		}
	}
	return copies;
}

/* Phase A for one device: sma.c:66-121 restricted to the given replicas.  */
int cbo_sma_accumulate (int R, size_t n, float alpha, const float *z,
		float **s, float **w, const int *copy, float *acc) {
	int i, copies = 0;
	size_t k;
	memset (acc, 0, n * sizeof(float));                                     /* sma.c:66 */
	for (i = 0; i < R; ++i) {
		for (k = 0; k < n; ++k) {
			float d = fmaf (-1.0f, z[k], s[i][k]);                          /* sma.c:79-90 */
			w[i][k] = fmaf (-alpha, d, w[i][k]);                            /* sma.c:93-99 */
			acc[k] = fmaf (alpha, d, acc[k]);                               /* sma.c:102-107 */
		}
		if (copy && copy[i])
			copies++;
	}
	return copies;
}

/* Phases C and D for one device: sma.c:148-174, 185-227. */
void cbo_sma_apply (int R, size_t n, float momentum, const float *D,
		float *z, float *last, float **w, int copy) {
	int i;
	size_t k;
	for (k = 0; k < n; ++k) {
		float Dg = D[k];
		if (momentum > 0) {
			Dg = fmaf (CBO_BASE_MOMENTUM, last[k], Dg);
			last[k] = Dg;
		}
		z[k] = fmaf (1.0f, Dg, z[k]);
	}
	if (copy)
		for (i = 0; i < R; ++i)
			memcpy (w[i], z, n * sizeof(float));
}

/* Replica optimiser step, clib-multigpu/kernels/optimisers/sma.cu:3-100.  */
void cbo_sma_optimise (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *s) {
	size_t k;
	for (k = 0; k < n; ++k) {
		float gk = g[k];
		if (wd > 0)
			gk = fmaf (wd, w[k], gk);                                       /* sma.cu:24-31 */
		if (momentum > 0) {
			gk = rate * gk;                                                 /* sma.cu:52-57 sscal */
			gk = fmaf (momentum, last[k], gk);                              /* sma.cu:58-64 */
			last[k] = gk;                                                   /* sma.cu:68    */
			s[k] = w[k];                                                    /* sma.cu:71    */
			w[k] = fmaf (1.0f, gk, w[k]);                                   /* sma.cu:74    */
		} else {
			s[k] = w[k];                                                    /* sma.cu:87    */
			w[k] = fmaf (rate, gk, w[k]);                                   /* sma.cu:90    */
		}
		g[k] = gk;
	}
}

/* ---------------------------------------------------------------------- */
/* OpenBLAS replay of the reference call sequence.                         */
/* ---------------------------------------------------------------------- */
typedef void (*saxpy_fn) (int, float, const float *, int, float *, int);
typedef void (*sscal_fn) (int, float, float *, int);
typedef void (*threads_fn) (int);

static void *blas_handle = NULL;
static saxpy_fn blas_saxpy = NULL;
static sscal_fn blas_sscal = NULL;
static threads_fn blas_threads = NULL;
static char blas_name[512] = "";

int cbo_blas_open (const char *path) {
	static const char *probe[] = { "libopenblas.so.0", "libopenblas.so", NULL };
	static const char *saxpy_names[] = { "cblas_saxpy", "scipy_cblas_saxpy", NULL };
	static const char *sscal_names[] = { "cblas_sscal", "scipy_cblas_sscal", NULL };
	static const char *thread_names[] = { "openblas_set_num_threads", "scipy_openblas_set_num_threads", NULL };
	int j;
	if (blas_handle)
		return 0;
	if (path)
		blas_handle = dlopen (path, RTLD_NOW | RTLD_LOCAL);
	for (j = 0; ! blas_handle && probe[j]; ++j) {
		blas_handle = dlopen (probe[j], RTLD_NOW | RTLD_LOCAL);
		if (blas_handle)
			path = probe[j];
	}
	if (! blas_handle)
		return -1;
	for (j = 0; ! blas_saxpy && saxpy_names[j]; ++j)
		blas_saxpy = (saxpy_fn) dlsym (blas_handle, saxpy_names[j]);
	for (j = 0; ! blas_sscal && sscal_names[j]; ++j)
		blas_sscal = (sscal_fn) dlsym (blas_handle, sscal_names[j]);
	for (j = 0; ! blas_threads && thread_names[j]; ++j)
		blas_threads = (threads_fn) dlsym (blas_handle, thread_names[j]);
	if (! blas_saxpy || ! blas_sscal) {
		dlclose (blas_handle);
		blas_handle = NULL;
		return -2;
	}
	snprintf (blas_name, sizeof(blas_name), "%s", path);
	/* clib-multigpu/BLAS.c:32: openblas_set_num_threads(1) */
	if (blas_threads)
		blas_threads (1);
	return 0;
}

const char *cbo_blas_name (void) { return blas_name; }

int cbo_blas_is_open (void) { return blas_handle != NULL; }

void cbo_blas_set_threads (int threads) {
	if (blas_threads)
		blas_threads (threads);
}

int cbo_sma_blas (int G, int size, size_t n, float alpha, float momentum,
		float **z, float **last, float **s, float **w,
		const int *locked, int *copy, int first, float *scratch) {

	int g, h, i, copies = 0;
	int N = (int) n; /* the reference passes model->elements, an int */
	size_t bytes = n * sizeof(float);
	float *gradient = scratch;                      /* base->gradient, per device */
	float *diff = scratch + (size_t) G * n;         /* base->diff, per device     */

	if (! blas_saxpy)
		return -1;

	for (g = 0; g < G; ++g) {
		float *acc = gradient + (size_t) g * n;
		float *d = diff + (size_t) g * n;
		memset (acc, 0, bytes);                                         /* sma.c:66 */
		for (i = first; i < size; ++i) {
			if (! locked[i] || (i % G) != g)
				continue;
			memcpy (d, s[i], bytes);                                    /* sma.c:79-83 */
			blas_saxpy (N, -1.0f, z[g], 1, d, 1);                       /* sma.c:85-90 */
			blas_saxpy (N, -alpha, d, 1, w[i], 1);                      /* sma.c:93-99 */
			blas_saxpy (N, alpha, d, 1, acc, 1);                        /* sma.c:102-107 */
			if (copy[i])
				copies++;
		}
	}

	/* common.c:43-52: receive buffer base->diff := all-reduce(base->gradient) */
	for (g = 0; g < G; ++g) {
		float *d = diff + (size_t) g * n;
		memcpy (d, gradient, bytes);
		for (h = 1; h < G; ++h)
			blas_saxpy (N, 1.0f, gradient + (size_t) h * n, 1, d, 1);
	}

	for (g = 0; g < G; ++g) {
		float *d = diff + (size_t) g * n;
		if (momentum > 0) {
			blas_saxpy (N, CBO_BASE_MOMENTUM, last[g], 1, d, 1);        /* sma.c:155-160 */
			memcpy (last[g], d, bytes);                                 /* sma.c:163-164 */
		}
		blas_saxpy (N, 1.0f, d, 1, z[g], 1);                            /* sma.c:169-174 */
	}

	if (copies > 0) {
		for (i = first; i < size; ++i) {
			if (! locked[i])
				continue;
			memcpy (w[i], z[i % G], bytes);                             /* sma.c:213-217 */
			copy[i] = 0;
		}
	}
	return copies;
}

/* sma.cu:3-100 as the reference issues it (cuBLAS -> OpenBLAS, memcpy).  */
int cbo_sma_optimise_blas (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *s) {
	int N = (int) n;
	size_t bytes = n * sizeof(float);
	if (! blas_saxpy || ! blas_sscal)
		return -1;
	if (wd > 0)
		blas_saxpy (N, wd, w, 1, g, 1);                                     /* sma.cu:24-31 */
	if (momentum > 0) {
		blas_sscal (N, rate, g, 1);                                         /* sma.cu:52-57 */
		blas_saxpy (N, momentum, last, 1, g, 1);                            /* sma.cu:58-64 */
		memcpy (last, g, bytes);                                            /* sma.cu:68    */
		memcpy (s, w, bytes);                                               /* sma.cu:71    */
		blas_saxpy (N, 1.0f, g, 1, w, 1);                                   /* sma.cu:74    */
	} else {
		memcpy (s, w, bytes);                                               /* sma.cu:87    */
		blas_saxpy (N, rate, g, 1, w, 1);                                   /* sma.cu:90    */
	}
	return 0;
}

/* ---------------------------------------------------------------------- */
/* DEFAULT (update model 0).                                               */
/* ---------------------------------------------------------------------- */
void cbo_default_task (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *z) {
	size_t k;
	for (k = 0; k < n; ++k) {
		float gk = g[k];
		if (wd > 0)
			gk = fmaf (wd, w[k], gk);                                       /* default.cu:26-35   */
		if (momentum > 0) {
			gk = rate * gk;                                                 /* default.cu:46-53 sscal */
			gk = fmaf (momentum, last[k], gk);                              /* default.cu:55-62   */
			last[k] = gk;                                                   /* default.cu:68-73   */
			w[k] = fmaf (1.0f, gk, w[k]);                                   /* default.cu:75-82   */
			z[k] = fmaf (1.0f, gk, z[k]);                                   /* default.cu:87-94   */
		} else {
			w[k] = fmaf (rate, gk, w[k]);                                   /* default.cu:106-113 */
			z[k] = fmaf (rate, gk, z[k]);                                   /* default.cu:118-125 */
		}
		g[k] = gk;
	}
}

int cbo_default_task_blas (size_t n, float rate, float momentum, float wd,
		float *w, float *g, float *last, float *z) {
	int N = (int) n;
	if (! blas_saxpy || ! blas_sscal)
		return -1;
	if (wd > 0)
		blas_saxpy (N, wd, w, 1, g, 1);
	if (momentum > 0) {
		blas_sscal (N, rate, g, 1);
		blas_saxpy (N, momentum, last, 1, g, 1);
		memcpy (last, g, n * sizeof(float));
		blas_saxpy (N, 1.0f, g, 1, w, 1);
		blas_saxpy (N, 1.0f, g, 1, z, 1);
	} else {
		blas_saxpy (N, rate, g, 1, w, 1);
		blas_saxpy (N, rate, g, 1, z, 1);
	}
	return 0;
}

void cbo_default_sync (int size, size_t n, const float *z, float **w, const int *locked, int first) {
	int i;
	for (i = first; i < size; ++i)
		if (locked[i])
			memcpy (w[i], z, n * sizeof(float));                           /* default.c:19-37 */
}

/* ---------------------------------------------------------------------- */
/* Synchronous SGD (WORKER).                                               */
/* ---------------------------------------------------------------------- */
void cbo_ssgd_worker (size_t n, float rate, float wd, const float *w, float *g, float *acc) {
	size_t k;
	for (k = 0; k < n; ++k) {
		float gk = g[k];
		if (wd > 0) {
			gk = fmaf (wd, w[k], gk);                                       /* synchronoussgd.cu:20-26 */
			g[k] = gk;
		}
		acc[k] = fmaf (rate, gk, acc[k]);                                   /* synchronoussgd.cu:46-52 */
	}
}

int cbo_ssgd_worker_blas (size_t n, float rate, float wd, const float *w, float *g, float *acc) {
	if (! blas_saxpy)
		return -1;
	if (wd > 0)
		blas_saxpy ((int) n, wd, w, 1, g, 1);
	blas_saxpy ((int) n, rate, g, 1, acc, 1);
	return 0;
}

static float ssgd_ratio (int wpc) {
	return (float) (1.0 / (double) (float) wpc);                            /* synchronoussgd.c:55 */
}

void cbo_ssgd_sync (int G, int size, size_t n, int wpc, float momentum,
		float **z, float **last, float **w, float **acc,
		const int *locked, int first, float *scratch) {
	int g, h, i;
	size_t k;
	float ratio = ssgd_ratio (wpc);
	float *D = scratch;
	memcpy (D, acc[0], n * sizeof(float));                                  /* common.c:43-52 */
	for (h = 1; h < G; ++h)
		for (k = 0; k < n; ++k)
			D[k] = D[k] + acc[h][k];
	for (g = 0; g < G; ++g) {
		for (k = 0; k < n; ++k) {
			float Dg = ratio * D[k];                                        /* synchronoussgd.c:55-62 */
			if (momentum > 0) {
				Dg = fmaf (momentum, last[g][k], Dg);                       /* :64-71 */
				last[g][k] = Dg;                                            /* :74-75 */
			}
			z[g][k] = fmaf (1.0f, Dg, z[g][k]);                             /* :79-84 */
		}
		memset (acc[g], 0, n * sizeof(float));                              /* :103 */
		for (i = first; i < size; ++i)
			if (locked[i] && (i % G) == g)
				memcpy (w[i], z[g], n * sizeof(float));                     /* common.c:206-214 */
	}
}

int cbo_ssgd_sync_blas (int G, int size, size_t n, int wpc, float momentum,
		float **z, float **last, float **w, float **acc,
		const int *locked, int first, float *scratch) {
	int g, h, i, N = (int) n;
	size_t bytes = n * sizeof(float);
	float ratio = ssgd_ratio (wpc);
	float *sum = scratch, *D = scratch + n;
	if (! blas_saxpy || ! blas_sscal)
		return -1;
	memcpy (sum, acc[0], bytes);
	for (h = 1; h < G; ++h)
		blas_saxpy (N, 1.0f, acc[h], 1, sum, 1);
	for (g = 0; g < G; ++g) {
		memcpy (D, sum, bytes);                                             /* base->diff of device g */
		blas_sscal (N, ratio, D, 1);
		if (momentum > 0) {
			blas_saxpy (N, momentum, last[g], 1, D, 1);
			memcpy (last[g], D, bytes);
		}
		blas_saxpy (N, 1.0f, D, 1, z[g], 1);
		memset (acc[g], 0, bytes);
		for (i = first; i < size; ++i)
			if (locked[i] && (i % G) == g)
				memcpy (w[i], z[g], bytes);
	}
	return 0;
}

/* ---------------------------------------------------------------------- */
/* Batch-norm statistics averaging, cudnn/cudnnbatchnormparams.c:157-222   */
/* ---------------------------------------------------------------------- */
int cbo_bn_average (int G, int layers, const int *elements, float **mean, float **var, const int *updated) {
	int l, g;
	size_t k;
	if (G == 1)                                                             /* :165-166 */
		return 0;
	for (l = 0; l < layers; ++l) {
		float *M = mean[l], *V = var[l];                                    /* default device 0 */
		size_t n = (size_t) elements[l];
		int count = 1;
		for (g = 1; g < G; ++g) {
			if (! updated[g * layers + l])                                  /* :175 */
				continue;
			for (k = 0; k < n; ++k) {
				M[k] = fmaf (1.0f, mean[g * layers + l][k], M[k]);           /* :185 */
				V[k] = fmaf (1.0f, var[g * layers + l][k], V[k]);            /* :186 */
			}
			count++;
		}
		if (count > 1) {                                                    /* :192-197 */
			float ratio = (float) (1. / (float) count);
			for (k = 0; k < n; ++k) {
				M[k] = ratio * M[k];
				V[k] = ratio * V[k];
			}
		}
		for (g = 1; g < G; ++g) {                                           /* :200-209 */
			memcpy (mean[g * layers + l], M, n * sizeof(float));
			memcpy (var[g * layers + l], V, n * sizeof(float));
		}
	}
	return 0;
}

/* ---------------------------------------------------------------------- */
/* CPU affinity, clib-multigpu/CPU.c:39-60                                 */
/* ---------------------------------------------------------------------- */
int cbo_bind_core (int core) {
	cpu_set_t set;
	CPU_ZERO (&set);
	CPU_SET (core, &set);
	return sched_setaffinity (0, sizeof(set), &set);
}

int cbo_unbind (void) {
	cpu_set_t set;
	long j, ncores = sysconf (_SC_NPROCESSORS_ONLN);
	CPU_ZERO (&set);
	for (j = 0; j < ncores && j < CPU_SETSIZE; ++j)
		CPU_SET (j, &set);
	return sched_setaffinity (0, sizeof(set), &set);
}

double cbo_now (void) {
	struct timespec ts;
	clock_gettime (CLOCK_MONOTONIC, &ts);
	return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

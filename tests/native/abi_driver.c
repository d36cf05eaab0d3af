/*
 * abi_driver.c -- drives libcrossbow_sma's C-ABI from plain C, the way the
 * JNI shim does, through every host-side path: registration, the model
 * manager, BSP/SSP barriers, SMA / S-SGD / DEFAULT steps, the optimiser
 * step, pinned staging (serial and pipelined), checkpoint / override (with
 * batch-norm statistics),
 * autotune add / del (also while task threads reserve, lock and release
 * replicas: the ids they hold may be deleted under them), BN averaging,
 * timing queries, one process over four (repeated) devices with the
 * per-device enqueue threads on and off, and teardown.
 *
 * Built with host-side AddressSanitizer + UndefinedBehaviorSanitizer
 * (scripts/build_sanitized.sh: -Xarch_host -fsanitize=..., GPU code is not
 * instrumented) and run on the GPU box by tests/test_gpu_sanitized.py.
 * Exit status 0 = every call returned as expected and the results are sane.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "crossbow_sma.h"

#define CHECK(call)                                                                  \
	do {                                                                             \
		int rc_ = (call);                                                            \
		if (rc_ < 0) {                                                               \
			fprintf (stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_,  \
				cbx_last_error ());                                                  \
			exit (1);                                                                \
		}                                                                            \
	} while (0)

#define EXPECT(cond)                                                                 \
	do {                                                                             \
		if (! (cond)) {                                                              \
			fprintf (stderr, "%s:%d expectation failed: %s\n", __FILE__, __LINE__, #cond); \
			exit (1);                                                                \
		}                                                                            \
	} while (0)

static cbx_context *setup_on (int ndev, int n1, int n2, int R, int sync, int type, float momentum) {
	cbx_context *c = NULL;
	int devs[4] = { 0, 0, 0, 0 };  /* one card repeated: the one-process form rehearsed */
	CHECK (cbx_init (&c, devs, ndev));
	int bytes = 4 * (n1 + n2);
	CHECK (cbx_set_model (c, 2, bytes));
	int s1[2] = { n1 / 4, 4 }, s2[1] = { n2 };
	CHECK (cbx_set_model_variable (c, 0, 1, 2, s1, 4 * n1));
	CHECK (cbx_set_model_variable (c, 1, 1, 1, s2, 4 * n2));
	float *init = malloc ((size_t) 4 * n1);
	for (int k = 0; k < n1; ++k) init[k] = 0.001f * (float) (k % 97);
	CHECK (cbx_set_model_variable_buffer (c, 0, 1, init));
	free (init);
	CHECK (cbx_set_model_work_per_clock (c, 2));
	CHECK (cbx_set_update_model_type (c, type));
	CHECK (cbx_set_learning_rate_decay_policy_fixed (c, 0.05f));
	CHECK (cbx_set_momentum (c, momentum, 0));
	CHECK (cbx_set_weight_decay (c, 1e-4f));
	CHECK (cbx_set_eamsgd_alpha (c, 0.1f));
	CHECK (cbx_set_model_manager (c, R, sync));
	EXPECT (cbx_num_replicas (c) == ndev * R);  /* R per device */
	EXPECT (cbx_model_elements (c) == n1 + n2);
	return c;
}

static cbx_context *setup (int n1, int n2, int R, int sync, int type, float momentum) {
	return setup_on (1, n1, n2, R, sync, type, momentum);
}

static void barrier (cbx_context *c, int clock, int autotune) {
	CHECK (cbx_lock_any (c));
	int first = -2;
	CHECK (cbx_merge (c, 0, &first));
	CHECK (cbx_synchronise (c, 0, clock, autotune, 0));
	CHECK (cbx_unlock_any (c));
}

static int all_finite (const float *p, size_t n) {
	for (size_t k = 0; k < n; ++k)
		if (! isfinite (p[k])) return 0;
	return 1;
}

/* Task threads against autotune: they reserve replicas through the theta
 * queue (acquireAccess / upgradeAccess, getNextOrWait), lock, release, while
 * the barrier thread adds and deletes one replica per device every step.
 * Calls on a deleted id may fail; nothing may touch freed memory (ASan). */
struct stress {
	cbx_context *c;
	atomic_int stop;
	atomic_long tasks;
};

static void *stress_task (void *arg) {
	struct stress *s = arg;
	int k = 0;
	while (! atomic_load (&s->stop)) {
		int clock = -1, id;
		if (k++ % 3 == 0) {
			id = cbx_get_next_or_wait (s->c, 0);  /* reserve + lock */
			if (id < 0) continue;
		} else {
			id = cbx_acquire_access (s->c, &clock);
			if (id < 0) continue;
			if (cbx_upgrade_access (s->c, id, &clock) != 1) continue;  /* deleted meanwhile */
			if (cbx_replica_lock (s->c, id) < 0) continue;
		}
		(void) cbx_replica_task_done (s->c, id);
		(void) cbx_replica_clock (s->c, id);
		(void) cbx_replica_release (s->c, id);  /* unlock + free the slot; fails on a deleted id */
		atomic_fetch_add (&s->tasks, 1);
	}
	return NULL;
}

static void stress_autotune (int n1, int n2) {
	struct stress s;
	s.c = setup (n1, n2, 2, CBX_SYNC_ASP, CBX_UPDATE_SMA, 0.9f);
	atomic_init (&s.stop, 0);
	atomic_init (&s.tasks, 0);
	pthread_t th[3];
	for (int t = 0; t < 3; ++t) EXPECT (pthread_create (&th[t], NULL, stress_task, &s) == 0);
	for (int clock = 1; clock <= 24; ++clock) {
		CHECK (cbx_lock_any (s.c));
		CHECK (cbx_synchronise (s.c, 0, clock, clock % 2 ? 1 : -1, 0));  /* add, then delete */
		CHECK (cbx_unlock_any (s.c));
		usleep (200);
	}
	atomic_store (&s.stop, 1);
	for (int t = 0; t < 3; ++t) EXPECT (pthread_join (th[t], NULL) == 0);
	EXPECT (cbx_num_replicas (s.c) == 2);
	EXPECT (atomic_load (&s.tasks) > 0);
	CHECK (cbx_wait (s.c));
	CHECK (cbx_free (s.c));
}

int main (void) {
	int count = 0;
	CHECK (cbx_device_count (&count));
	EXPECT (count >= 1);
	const int n1 = 40000, n2 = 3331, n = n1 + n2, R = 3;
	float *host = malloc ((size_t) 4 * n);

	/* SMA, BSP, momentum: tasks, barriers, staging, checkpoint, autotune */
	cbx_context *c = setup (n1, n2, R, CBX_SYNC_BSP, CBX_UPDATE_SMA, 0.9f);
	CHECK (cbx_fill_synthetic (c, 7));
	CHECK (cbx_set_timing (c, 1));
	for (int clock = 1; clock <= 3; ++clock) {
		for (int i = 0; i < R; ++i) {
			CHECK (cbx_replica_lock (c, i));
			CHECK (cbx_replica_optimise (c, i, clock * R + i, NULL));
			CHECK (cbx_replica_task_done (c, i));
			CHECK (cbx_replica_unlock (c, i));
		}
		barrier (c, clock, 0);
	}
	float ms[CBX_T_COUNT];
	CHECK (cbx_last_timing (c, 0, ms));
	EXPECT (ms[CBX_T_STEP] > 0);
	float hist[16];
	EXPECT (cbx_timing_history (c, 0, CBX_T_KERNEL, hist, 16) >= 3);
	void *ev = NULL;
	CHECK (cbx_step_event (c, 0, &ev));
	EXPECT (ev != NULL);
	CHECK (cbx_stage_out (c));
	CHECK (cbx_stage_in (c));
	CHECK (cbx_lock_any (c));
	CHECK (cbx_synchronise_staged (c, 0, 4, 0, 5));
	CHECK (cbx_unlock_any (c));
	CHECK (cbx_wait (c));
	void *hz = NULL;
	CHECK (cbx_base_host_buffer (c, 0, CBX_BUF_DATA, &hz));
	EXPECT (all_finite ((const float *) hz, (size_t) n));
	char dir[] = "/tmp/cbx_abi_driverXXXXXX";
	EXPECT (mkdtemp (dir) != NULL);
	{	/* one BN operator's statistics travel with the checkpoint */
		void *bn = NULL;
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_GRADIENT, &bn));
		float *bm[1] = { (float *) bn }, *bv[1] = { (float *) bn + 256 };
		CHECK (cbx_register_batchnorm_stats (c, 4, 256, bm, bv));
		float *half[1] = { NULL };
		EXPECT (cbx_register_batchnorm_stats (c, 5, 256, bm, half) == CBX_ERR_INVALID);
	}
	CHECK (cbx_checkpoint_model (c, dir));
	CHECK (cbx_base_read (c, 0, CBX_BUF_DATA, host, (size_t) 4 * n));
	barrier (c, 5, 1);  /* autotune: add one replica per device */
	EXPECT (cbx_num_replicas (c) == R + 1);
	barrier (c, 6, -1); /* and delete it again */
	EXPECT (cbx_num_replicas (c) == R);
	/* override from the checkpoint written above (its numbered subdirectory) */
	int rc = cbx_override_model_data (c, dir);
	(void) rc;  /* the directory layout is checked by the Python tests; here: no crash */
	float *z2 = malloc ((size_t) 4 * n);
	CHECK (cbx_base_read (c, 0, CBX_BUF_DATA, z2, (size_t) 4 * n));
	EXPECT (all_finite (z2, (size_t) n));
	free (z2);
	/* error paths keep the context usable */
	EXPECT (cbx_replica_lock (c, 99) == CBX_ERR_INVALID);
	EXPECT (cbx_synchronise_staged (c, 0, 7, 0, 0) == CBX_ERR_INVALID);
	EXPECT (cbx_set_kernel_config (c, 96, 0, 1, 1) == CBX_ERR_INVALID);
	{	/* the per-rank peer-read form's handles: one process over its devices has none to export */
		unsigned char blob[CBX_PEER_BLOB_BYTES];
		size_t bytes = 0;
		EXPECT (cbx_peer_export (c, blob, &bytes) == CBX_ERR_UNSUPPORTED);
		EXPECT (cbx_peer_import (c, blob, 1) == CBX_ERR_STATE);
	}
	CHECK (cbx_set_kernel_config (c, 64, 0, 1, 2));
	CHECK (cbx_set_aux_kernel_config (c, 128, 2, 4));
	barrier (c, 7, 0);
	/* the theta queue: reserve, run, release (modelmanager.c:147-204) */
	{
		int clk = -1;
		int a = cbx_acquire_access (c, &clk), b = cbx_acquire_access (c, &clk);
		EXPECT (a >= 0 && b >= 0 && a != b && clk >= 0);
		EXPECT (cbx_upgrade_access (c, a, &clk) == 1);
		EXPECT (cbx_replica_set_disabled (c, a, 1) == 1);  /* reserved: stays enabled */
		CHECK (cbx_replica_lock (c, a));
		CHECK (cbx_replica_release (c, a));
		CHECK (cbx_replica_lock (c, b));
		CHECK (cbx_replica_release (c, b));
		EXPECT (cbx_replica_release (c, b) == CBX_ERR_STATE);
		int d = cbx_get_next_or_wait (c, 0);
		EXPECT (d >= 0);
		CHECK (cbx_replica_release (c, d));
	}
	/* BSP failure: a replica held by a task */
	CHECK (cbx_replica_lock (c, 1));
	EXPECT (cbx_lock_any (c) == CBX_ERR_BARRIER);
	CHECK (cbx_replica_unlock (c, 1));
	CHECK (cbx_replica_set_disabled (c, 2, 1));
	EXPECT (cbx_lock_any (c) == R);
	CHECK (cbx_synchronise (c, 0, 8, 0, 0));
	EXPECT (cbx_unlock_any (c) == R - 1);
	CHECK (cbx_free (c));

	/* split pipeline over a one-rank communicator, SSP */
	c = setup (n1, n2, R, CBX_SYNC_SSP, CBX_UPDATE_SYNCHRONOUSEAMSGD, 0.9f);
	CHECK (cbx_set_force_split (c, 1));
	CHECK (cbx_set_bucket_elements (c, 8192));
	CHECK (cbx_replica_lock (c, 0));
	EXPECT (cbx_lock_any (c) == R - 1);
	CHECK (cbx_synchronise (c, 0, 1, 0, 0));
	CHECK (cbx_unlock_any (c));
	CHECK (cbx_replica_unlock (c, 0));
	CHECK (cbx_lock_any (c));
	CHECK (cbx_synchronise_staged (c, 0, 2, 0, 3));
	CHECK (cbx_unlock_any (c));
	CHECK (cbx_set_pipeline_mode (c, 1));  /* across steps */
	EXPECT (cbx_set_pipeline_mode (c, 2) == CBX_ERR_INVALID);
	EXPECT (cbx_set_pipeline_mode (c, -1) == CBX_ERR_INVALID);
	EXPECT (cbx_set_cross_wait_stride (c, 0) == CBX_ERR_INVALID);
	EXPECT (cbx_check_order (c) == CBX_ERR_STATE);  /* not enabled */
	EXPECT (cbx_set_allreduce_algorithm (c, 3) == CBX_ERR_INVALID);
	EXPECT (cbx_set_enqueue_threads (c, 2) == CBX_ERR_INVALID);
	EXPECT (cbx_set_enqueue_threads (c, -2) == CBX_ERR_INVALID);
	CHECK (cbx_set_enqueue_threads (c, 1));  /* one device: a pool of one thread */
	for (int clock = 3; clock < 13; ++clock) {
		if (clock == 5) CHECK (cbx_replica_set_copy (c, 1, 1));
		if (clock == 6) CHECK (cbx_set_pipeline_mode (c, 0));  /* back to within-step buckets */
		if (clock == 7) CHECK (cbx_set_cross_wait_stride (c, 3));
		if (clock == 8) CHECK (cbx_set_order_check (c, 1));
		if (clock == 9) CHECK (cbx_set_pipeline_mode (c, 1));
		if (clock == 10) CHECK (cbx_set_allreduce_algorithm (c, CBX_ALLREDUCE_RSAG));
		if (clock == 12) CHECK (cbx_set_order_check (c, 0));
		CHECK (cbx_lock_any (c));
		CHECK (cbx_synchronise (c, 0, clock, 0, 0));
		CHECK (cbx_unlock_any (c));
		if (clock == 9 || clock == 11) EXPECT (cbx_check_order (c) == 2);
	}
	CHECK (cbx_wait (c));
	CHECK (cbx_free (c));

	/* S-SGD (WORKER) and DEFAULT, no momentum */
	for (int type = 0; type < 2; ++type) {
		c = setup (n1, n2, R, CBX_SYNC_BSP, type == 0 ? CBX_UPDATE_WORKER : CBX_UPDATE_DEFAULT, 0.0f);
		for (int i = 0; i < R; ++i)
			CHECK (cbx_replica_optimise (c, i, i, NULL));
		barrier (c, 1, 0);
		CHECK (cbx_replica_read (c, 1, CBX_BUF_DATA, host, (size_t) 4 * n));
		EXPECT (all_finite (host, (size_t) n));
		CHECK (cbx_free (c));
	}

	stress_autotune (n1, n2);

	/* The sma.c seam over buffers the caller owns (here a context's, used as
	 * plain device memory), ragged so the tail kernel runs, Phase D asked. */
	c = setup (n1, n2, 2, CBX_SYNC_BSP, CBX_UPDATE_SMA, 0.9f);
	{
		const long long m = (long long) n - 5;
		void *z = NULL, *last = NULL, *w0 = NULL, *w1 = NULL, *s0 = NULL, *s1 = NULL, *g = NULL, *lr = NULL;
		CHECK (cbx_base_buffer (c, 0, CBX_BUF_DATA, &z));
		CHECK (cbx_base_buffer (c, 0, CBX_BUF_LAST, &last));
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_DATA, &w0));
		CHECK (cbx_replica_buffer (c, 1, CBX_BUF_DATA, &w1));
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_DIFF, &s0));
		CHECK (cbx_replica_buffer (c, 1, CBX_BUF_DIFF, &s1));
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_GRADIENT, &g));
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_LAST, &lr));
		cbx_sma_plan *plan = NULL;
		int dev = 0;
		CHECK (cbx_sma_plan_create (&plan, &dev, 1, m, NULL));
		void *streams[1] = { NULL };
		float *zz[1] = { (float *) z }, *ll[1] = { (float *) last }, *ww[2] = { (float *) w0, (float *) w1 };
		const float *ss[2] = { (const float *) s0, (const float *) s1 };
		int rdev[2] = { 0, 0 }, locked[2] = { 1, 1 }, copy[2] = { 0, 1 };
		CHECK (cbx_sma_optimise_buffers (NULL, (float *) w0, (float *) g, (float *) lr, (float *) s0, m, 0.05f, 0.9f,
			1e-4f));
		EXPECT (cbx_sma_plan_step (plan, streams, zz, ll, 2, rdev, ww, ss, locked, copy, 0.1f, 0.9f, 0) == 1);
		copy[1] = 0;
		EXPECT (cbx_sma_plan_step (plan, streams, zz, ll, 2, rdev, ww, ss, locked, copy, 0.1f, 0.9f, 1) == 0);
		EXPECT (cbx_sma_plan_step (plan, streams, zz, ll, 2, rdev, ww, ss, locked, copy, 0.1f, 0.9f, 3) == CBX_ERR_INVALID);
		EXPECT (cbx_sma_plan_step (plan, streams, zz, NULL, 2, rdev, ww, ss, locked, copy, 0.1f, 0.9f, 0) == CBX_ERR_INVALID);
		/* the S-SGD seam: a task step into the base gradient, then the barrier */
		void *acc = NULL;
		CHECK (cbx_base_buffer (c, 0, CBX_BUF_GRADIENT, &acc));
		float *aa[1] = { (float *) acc };
		CHECK (cbx_ssgd_accumulate_buffers (NULL, (const float *) w0, (float *) g, (float *) acc, m, 0.05f, 1e-4f));
		CHECK (cbx_ssgd_plan_step (plan, streams, zz, ll, aa, 2, rdev, ww, locked, 0.9f, 4, 0));
		EXPECT (cbx_ssgd_plan_step (plan, streams, zz, ll, aa, 2, rdev, ww, locked, 0.9f, 0, 0) == CBX_ERR_INVALID);
		CHECK (cbx_sma_plan_free (plan));
		CHECK (cbx_replica_read (c, 0, CBX_BUF_DATA, host, (size_t) 4 * n));
		EXPECT (all_finite (host, (size_t) m));
		EXPECT (cbx_sma_plan_create (&plan, &dev, 1, 0, NULL) == CBX_ERR_INVALID);
	}
	CHECK (cbx_free (c));

	/* BN statistics averaging is a no-op with one device but walks its tables */
	c = setup (n1, n2, 1, CBX_SYNC_BSP, CBX_UPDATE_SMA, 0.0f);
	{
		void *p = NULL;
		CHECK (cbx_replica_buffer (c, 0, CBX_BUF_GRADIENT, &p));
		float *mean[2] = { (float *) p, (float *) p + 64 };
		float *var[2] = { (float *) p + 128, (float *) p + 192 };
		int elements[2] = { 64, 64 }, updated[2] = { 1, 1 };
		CHECK (cbx_average_batchnorm_stats (c, 2, elements, mean, var, updated));
	}
	CHECK (cbx_free (c));

	/* One process over several devices (the card repeated, so peer reads):
	 * each device's step enqueued by its own pool thread, then by this one,
	 * within-step and cross-step buckets, the pool torn down by cbx_free. */
	for (int threads = 1; threads >= 0; --threads) {
		c = setup_on (4, n1, n2, 1, CBX_SYNC_BSP, CBX_UPDATE_SMA, 0.9f);
		CHECK (cbx_set_allreduce_algorithm (c, CBX_ALLREDUCE_PEER));
		CHECK (cbx_set_enqueue_threads (c, threads));
		CHECK (cbx_set_bucket_elements (c, 4096));
		for (int clock = 1; clock < 9; ++clock) {
			if (clock == 4) CHECK (cbx_set_pipeline_mode (c, 1));
			if (clock == 6) CHECK (cbx_set_timing (c, 1));  /* span records: G x 2 waits per reduction */
			CHECK (cbx_lock_any (c));
			CHECK (cbx_synchronise (c, 0, clock, 0, 0));
			CHECK (cbx_unlock_any (c));
		}
		CHECK (cbx_wait (c));
		{
			float ms[CBX_T_COUNT], hist[8];
			CHECK (cbx_last_timing (c, 3, ms));
			EXPECT (cbx_timing_history (c, 0, CBX_T_ALLREDUCE, hist, 8) == 3);
		}
		CHECK (cbx_replica_read (c, 3, CBX_BUF_DATA, host, (size_t) 4 * n));
		EXPECT (all_finite (host, (size_t) n));
		CHECK (cbx_free (c));
	}
	free (host);
	printf ("abi_driver: ok\n");
	fflush (stdout);
	/* Every context is freed above.  Skip the HIP runtime's own static
	 * teardown: under host ASan it can trip ASan's device-allocator check
	 * ("dev_runtime_unloaded_") in libhsa-runtime64's destructors, which
	 * is not this library's code. */
	_exit (0);
}

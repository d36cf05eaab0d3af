/*
 * TheGPU_jni.c -- JNI shim exporting Crossbow's TheGPU model-path natives on
 * top of libcrossbow_sma.so.  Built by crossbow_amd/build.py only where a JDK
 * provides jni.h (none in this image).
 *
 * Signatures follow clib-multigpu/uk_ac_imperial_lsds_crossbow_device_TheGPU.h
 * (e.g. synchronise (IIIZ)I at :636-640).  Like the reference (static theGPU,
 * GPU.c:12) the context is process-global, and like the reference every
 * failure prints to stderr and exits (debug.h:37-57).
 */
#include <jni.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crossbow_sma.h"

static cbx_context *theGPU = NULL;

/* The dataflow natives that stay in the reference's GPU.c (execute, the
 * callback handler, ...) are linked into the same libGPU.so and reach the
 * model manager through this context (cbx_replica_lock / _release /
 * _buffer / _optimise, ...).  Declare it there as
 *     extern cbx_context *crossbow_sma_context (void);                    */
cbx_context *crossbow_sma_context (void);
cbx_context *crossbow_sma_context (void) {
	return theGPU;
}

static jint fatal_or (int rc) {
	if (rc < 0) {
		fprintf (stderr, "error: %s\n", cbx_last_error ());
		exit (1);
	}
	return (jint) rc;
}

#define NATIVE(ret, name) JNIEXPORT ret JNICALL Java_uk_ac_imperial_lsds_crossbow_device_TheGPU_##name

/* The Java side has no natives for this library's G > 1 pipeline settings
 * (Crossbow's own step is one grouped all-reduce), so a deployment chooses
 * them through the environment, read once at init (values as the C-ABI
 * takes them; an unparsable or refused value is fatal, like every error):
 *   CBX_ALLREDUCE          rccl | rsag | peer   (cbx_set_allreduce_algorithm)
 *   CBX_BUCKET_ELEMENTS    floats per bucket    (cbx_set_bucket_elements)
 *   CBX_PIPELINE_MODE      0 | 1                (cbx_set_pipeline_mode)
 *   CBX_CROSS_WAIT_STRIDE  1..4096              (cbx_set_cross_wait_stride)
 *   CBX_ALLREDUCE_GROUP    1..4096              (cbx_set_allreduce_group)
 *   CBX_STAGING            zerocopy | dma       (cbx_set_staging_mode)
 *   CBX_ENQUEUE_THREADS    -1 | 0 | 1           (cbx_set_enqueue_threads)
 * bench.py's warm-up tuner (crossbow_amd/dist.py) prints the values it
 * chose for a node in its JSON config. */
static long long env_int (const char *name, int *present) {
	const char *v = getenv (name);
	*present = v != NULL && *v != '\0';
	if (!*present)
		return 0;
	char *end = NULL;
	long long x = strtoll (v, &end, 10);
	if (end == v || *end != '\0') {
		fprintf (stderr, "error: %s=%s is not an integer\n", name, v);
		exit (1);
	}
	return x;
}

static void configure_from_env (void) {
	const char *algo = getenv ("CBX_ALLREDUCE");
	if (algo && *algo) {
		int a = !strcmp (algo, "rccl") ? CBX_ALLREDUCE_RCCL : !strcmp (algo, "rsag") ? CBX_ALLREDUCE_RSAG
			: !strcmp (algo, "peer") ? CBX_ALLREDUCE_PEER : -1;
		if (a < 0) {
			fprintf (stderr, "error: CBX_ALLREDUCE=%s (rccl, rsag or peer)\n", algo);
			exit (1);
		}
		fatal_or (cbx_set_allreduce_algorithm (theGPU, a));
	}
	const char *staging = getenv ("CBX_STAGING");
	if (staging && *staging) {
		int m = !strcmp (staging, "zerocopy") ? CBX_STAGING_ZEROCOPY : !strcmp (staging, "dma") ? CBX_STAGING_DMA : -1;
		if (m < 0) {
			fprintf (stderr, "error: CBX_STAGING=%s (zerocopy or dma)\n", staging);
			exit (1);
		}
		fatal_or (cbx_set_staging_mode (theGPU, m));
	}
	int on;
	long long v = env_int ("CBX_BUCKET_ELEMENTS", &on);
	if (on) fatal_or (cbx_set_bucket_elements (theGPU, v));
	/* the int settings: out-of-range values go to the setter as -1 (refused) */
	v = env_int ("CBX_PIPELINE_MODE", &on);
	if (on) fatal_or (cbx_set_pipeline_mode (theGPU, v < 0 || v > 4096 ? -1 : (int) v));
	v = env_int ("CBX_CROSS_WAIT_STRIDE", &on);
	if (on) fatal_or (cbx_set_cross_wait_stride (theGPU, v < 0 || v > 4096 ? -1 : (int) v));
	v = env_int ("CBX_ALLREDUCE_GROUP", &on);
	if (on) fatal_or (cbx_set_allreduce_group (theGPU, v < 0 || v > 4096 ? -1 : (int) v));
	v = env_int ("CBX_ENQUEUE_THREADS", &on);
	if (on) fatal_or (cbx_set_enqueue_threads (theGPU, v < -1 || v > 1 ? -2 : (int) v));
}

/* GPU.c:21-63.  Thread-count / core-offset arguments configure the reference's
 * task and callback handler threads, which are not on this path. */
NATIVE(jint, init) (JNIEnv *env, jobject obj, jintArray devices, jint streams, jint callbacks,
		jint tasks, jint cboffset, jint tkoffset) {
	(void) obj; (void) streams; (void) callbacks; (void) tasks; (void) cboffset; (void) tkoffset;
	if (theGPU) {
		fprintf (stderr, "error: GPU execution context already initialised\n");
		exit (1);
	}
	jsize argc = (*env)->GetArrayLength (env, devices);
	jint *argv = (*env)->GetIntArrayElements (env, devices, 0);
	int rc = cbx_init (&theGPU, (const int *) argv, (int) argc);
	(*env)->ReleaseIntArrayElements (env, devices, argv, JNI_ABORT);
	fatal_or (rc);
	configure_from_env ();
	return 0;
}

NATIVE(jint, free) (JNIEnv *env, jobject obj) {
	(void) env; (void) obj;
	int rc = cbx_free (theGPU);
	theGPU = NULL;
	return fatal_or (rc);
}

NATIVE(jint, setModel) (JNIEnv *env, jobject obj, jint variables, jint size) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_model (theGPU, variables, size));
}

NATIVE(jint, setModelVariable) (JNIEnv *env, jobject obj, jint id, jint order, jintArray dims, jint capacity) {
	(void) obj;
	jsize argc = (*env)->GetArrayLength (env, dims);
	jint *argv = (*env)->GetIntArrayElements (env, dims, 0);
	int rc = cbx_set_model_variable (theGPU, id, order, (int) argc, (const int *) argv, capacity);
	(*env)->ReleaseIntArrayElements (env, dims, argv, JNI_ABORT);
	return fatal_or (rc);
}

NATIVE(jint, setModelVariableBuffer) (JNIEnv *env, jobject obj, jint id, jint order, jobject buffer) {
	(void) obj;
	return fatal_or (cbx_set_model_variable_buffer (theGPU, id, order, (*env)->GetDirectBufferAddress (env, buffer)));
}

NATIVE(jint, setModelVariableLearningRateMultiplier) (JNIEnv *env, jobject obj, jint id, jint order, jfloat multiplier) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_model_variable_learning_rate_multiplier (theGPU, id, order, multiplier));
}

NATIVE(jint, setModelWorkPerClock) (JNIEnv *env, jobject obj, jint wpc) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_model_work_per_clock (theGPU, wpc));
}

NATIVE(jint, setUpdateModelType) (JNIEnv *env, jobject obj, jint type) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_update_model_type (theGPU, type));
}

NATIVE(jint, setLearningRateDecayPolicyFixed) (JNIEnv *env, jobject obj, jfloat rate) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_learning_rate_decay_policy_fixed (theGPU, rate));
}

NATIVE(jint, setLearningRateDecayPolicyInv) (JNIEnv *env, jobject obj, jfloat rate, jdouble gamma, jdouble power) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_learning_rate_decay_policy_inv (theGPU, rate, gamma, power));
}

NATIVE(jint, setLearningRateDecayPolicyStep) (JNIEnv *env, jobject obj, jfloat rate, jdouble gamma, jint size) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_learning_rate_decay_policy_step (theGPU, rate, gamma, size));
}

NATIVE(jint, setLearningRateDecayPolicyMultiStep) (JNIEnv *env, jobject obj, jfloat rate, jdouble gamma,
		jint warmup, jintArray steps) {
	(void) obj;
	jsize argc = (*env)->GetArrayLength (env, steps);
	jint *argv = (*env)->GetIntArrayElements (env, steps, 0);
	int rc = cbx_set_learning_rate_decay_policy_multistep (theGPU, rate, gamma, warmup, (int) argc, (const int *) argv);
	(*env)->ReleaseIntArrayElements (env, steps, argv, JNI_ABORT);
	return fatal_or (rc);
}

NATIVE(jint, setLearningRateDecayPolicyExp) (JNIEnv *env, jobject obj, jfloat rate, jdouble gamma) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_learning_rate_decay_policy_exp (theGPU, rate, gamma));
}

/* GPU.c:803-822 */
NATIVE(jint, setLearningRateDecayPolicyCircular) (JNIEnv *env, jobject obj, jfloatArray rate, jint superconvergence,
		jfloatArray momentum, jint step) {
	(void) obj;
	if ((*env)->GetArrayLength (env, rate) != 3 || (*env)->GetArrayLength (env, momentum) != 3) {
		fprintf (stderr, "error: circular learning rate policy needs 3 rates and 3 momenta\n");
		exit (1);
	}
	jfloat *H = (*env)->GetFloatArrayElements (env, rate, 0);
	jfloat *M = (*env)->GetFloatArrayElements (env, momentum, 0);
	int rc = cbx_set_learning_rate_decay_policy_circular (theGPU, (const float *) H, superconvergence,
			(const float *) M, step);
	(*env)->ReleaseFloatArrayElements (env, rate, H, JNI_ABORT);
	(*env)->ReleaseFloatArrayElements (env, momentum, M, JNI_ABORT);
	return fatal_or (rc);
}

NATIVE(jint, setBaseModelMomentum) (JNIEnv *env, jobject obj, jfloat momentum) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_base_model_momentum (theGPU, momentum));
}

NATIVE(jint, setMomentum) (JNIEnv *env, jobject obj, jfloat momentum, jint method) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_momentum (theGPU, momentum, method));
}

NATIVE(jint, setWeightDecay) (JNIEnv *env, jobject obj, jfloat decay) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_weight_decay (theGPU, decay));
}

NATIVE(jint, setEamsgdAlpha) (JNIEnv *env, jobject obj, jfloat alpha) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_eamsgd_alpha (theGPU, alpha));
}

NATIVE(jint, setEamsgdTau) (JNIEnv *env, jobject obj, jint tau) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_eamsgd_tau (theGPU, tau));
}

NATIVE(jint, setModelManager) (JNIEnv *env, jobject obj, jint replicas, jint type) {
	(void) env; (void) obj;
	return fatal_or (cbx_set_model_manager (theGPU, replicas, type));
}

/* GPU.c:1113-1120; executioncontext.c:2199-2205 exits when BSP cannot lock all. */
NATIVE(jint, lockAny) (JNIEnv *env, jobject obj) {
	(void) env; (void) obj;
	return fatal_or (cbx_lock_any (theGPU));
}

NATIVE(jint, merge) (JNIEnv *env, jobject obj, jboolean pull) {
	(void) env; (void) obj;
	int first = -1;
	fatal_or (cbx_merge (theGPU, pull == JNI_TRUE ? 1 : 0, &first));
	return (jint) first;
}

NATIVE(jint, synchronise) (JNIEnv *env, jobject obj, jint first, jint clock, jint autotune, jboolean push) {
	(void) env; (void) obj;
	return fatal_or (cbx_synchronise (theGPU, first, clock, autotune, push == JNI_TRUE ? 1 : 0));
}

/* Not in the reference: the pipelined host-staged step (cbx_synchronise_staged).
 * Java side: `public native int synchroniseStaged (int first, int clock,
 * int autotune, int buckets);` next to synchronise (TheGPU.java:346). */
NATIVE(jint, synchroniseStaged) (JNIEnv *env, jobject obj, jint first, jint clock, jint autotune, jint buckets) {
	(void) env; (void) obj;
	return fatal_or (cbx_synchronise_staged (theGPU, first, clock, autotune, buckets));
}

NATIVE(jint, unlockAny) (JNIEnv *env, jobject obj) {
	(void) env; (void) obj;
	return fatal_or (cbx_unlock_any (theGPU));
}

NATIVE(jint, checkpointModel) (JNIEnv *env, jobject obj, jstring dir) {
	(void) obj;
	const char *path = (*env)->GetStringUTFChars (env, dir, NULL);
	int rc = cbx_checkpoint_model (theGPU, path);
	(*env)->ReleaseStringUTFChars (env, dir, path);
	return fatal_or (rc);
}

NATIVE(jint, overrideModelData) (JNIEnv *env, jobject obj, jstring dir) {
	(void) obj;
	if ((*env)->IsSameObject (env, dir, NULL))
		return 0; /* GPU.c:1169 */
	const char *path = (*env)->GetStringUTFChars (env, dir, NULL);
	int rc = cbx_override_model_data (theGPU, path);
	(*env)->ReleaseStringUTFChars (env, dir, path);
	return fatal_or (rc);
}

NATIVE(jint, addModel) (JNIEnv *env, jobject obj) {
	(void) env; (void) obj;
	return fatal_or (cbx_add_model (theGPU));
}

NATIVE(jint, delModel) (JNIEnv *env, jobject obj) {
	(void) env; (void) obj;
	return fatal_or (cbx_del_model (theGPU));
}

/* The theta queue (GPU.c:888-932 -> modelmanager.c:180-198).  Replica ids
 * cross JNI as java.lang.Integer, as in the reference (modelmanager.c:187). */
static jobject box (JNIEnv *env, int id) {
	jclass cls = (*env)->FindClass (env, "java/lang/Integer");
	jmethodID valueOf = (*env)->GetStaticMethodID (env, cls, "valueOf", "(I)Ljava/lang/Integer;");
	return (*env)->CallStaticObjectMethod (env, cls, valueOf, (jint) id);
}

static int unbox (JNIEnv *env, jobject obj) {
	jclass cls = (*env)->FindClass (env, "java/lang/Integer");
	jmethodID intValue = (*env)->GetMethodID (env, cls, "intValue", "()I");
	return (int) (*env)->CallIntMethod (env, obj, intValue);
}

static int *clock_arg (JNIEnv *env, jintArray clock, jint **argv) {
	if ((*env)->GetArrayLength (env, clock) != 1) { /* GPU.c:897 */
		fprintf (stderr, "error: clock must be an int[1]\n");
		exit (1);
	}
	*argv = (*env)->GetIntArrayElements (env, clock, 0);
	return (int *) *argv;
}

NATIVE(jobject, acquireAccess) (JNIEnv *env, jobject obj, jintArray clock) {
	(void) obj;
	jint *argv;
	int *c = clock_arg (env, clock, &argv);
	int id = (int) fatal_or (cbx_acquire_access (theGPU, c));
	(*env)->ReleaseIntArrayElements (env, clock, argv, 0);
	return box (env, id);
}

NATIVE(jobject, upgradeAccess) (JNIEnv *env, jobject obj, jobject replicaId, jintArray clock) {
	(void) obj;
	if ((*env)->IsSameObject (env, replicaId, NULL))
		return NULL;
	jint *argv;
	int *c = clock_arg (env, clock, &argv);
	int held = (int) fatal_or (cbx_upgrade_access (theGPU, unbox (env, replicaId), c));
	(*env)->ReleaseIntArrayElements (env, clock, argv, 0);
	return held ? replicaId : NULL;
}

NATIVE(jint, release) (JNIEnv *env, jobject obj, jobject replicaId) {
	(void) env; (void) obj; (void) replicaId;
	fprintf (stderr, "error: Cannot release a GPU model replica id object from the GPU\n"); /* GPU.c:930 */
	exit (1);
}

/*
 * jni_driver.c -- TEST INFRASTRUCTURE: calls the JNI shim's TheGPU natives
 * (crossbow_amd/csrc/jni/TheGPU_jni.c) in the order Crossbow's Java side does
 * (Model.GPURegister, SolverConf.GPURegister, ModelManager, TaskProcessor,
 * ResultCollector), with a hand-made JNIEnv standing in for a JVM: arrays,
 * direct buffers, strings and java.lang.Integer boxes are plain C objects.
 * The shim is compiled against tests/jni_stub/jni.h for this (no JDK here);
 * scripts/build_jni_harness.sh builds both.  tests/test_gpu_jni.py runs it
 * on the GPU box.
 *
 * Checks: the model registered through setModelVariableBuffer, one SMA step
 * through lockAny / merge / synchronise / unlockAny, written by
 * checkpointModel in the reference's file format, equals the oracle
 * (oracle/sma_oracle.c) bit for bit; overrideModelData restores it;
 * acquireAccess / upgradeAccess hand out replicas round robin as boxed
 * Integers; addModel / delModel; free.  Exit 0 = pass.
 *
 * `jni_driver G` runs the same sequence over G devices in one process (the
 * reference's own multi-GPU form, executioncontext.c:185-201): init gets G
 * copies of device 0, so this needs the library build linked against the
 * loopback collective (scripts/build_fake_rccl.sh builds that variant as
 * tests/native/jni_driver_fakerccl); the checkpoint then holds one set of
 * files per device, each checked against the oracle run with the same G.
 */
#define _GNU_SOURCE
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <jni.h>

#include "crossbow_sma.h"
#include "sma_oracle.h"

/* ---- a JVM's worth of objects ----------------------------------------- */
enum { OBJ_INT_ARRAY, OBJ_FLOAT_ARRAY, OBJ_BUFFER, OBJ_STRING, OBJ_INTEGER, OBJ_CLASS };
struct _jobject {
	int kind;
	jint len;
	void *data;
	jint value;
};
struct _jmethodID {
	int dummy;
};

static struct _jobject integer_class = { OBJ_CLASS, 0, NULL, 0 };
static struct _jmethodID method = { 0 };
static int boxes = 0;

static jsize f_GetArrayLength (JNIEnv *env, jobject o) { (void) env; return o->len; }
static jint *f_GetIntArrayElements (JNIEnv *env, jintArray a, jboolean *c) {
	(void) env; if (c) *c = JNI_FALSE; return (jint *) a->data;
}
static void f_ReleaseIntArrayElements (JNIEnv *env, jintArray a, jint *p, jint mode) {
	(void) env; (void) a; (void) p; (void) mode;
}
static jfloat *f_GetFloatArrayElements (JNIEnv *env, jfloatArray a, jboolean *c) {
	(void) env; if (c) *c = JNI_FALSE; return (jfloat *) a->data;
}
static void f_ReleaseFloatArrayElements (JNIEnv *env, jfloatArray a, jfloat *p, jint mode) {
	(void) env; (void) a; (void) p; (void) mode;
}
static void *f_GetDirectBufferAddress (JNIEnv *env, jobject b) { (void) env; return b->data; }
static const char *f_GetStringUTFChars (JNIEnv *env, jstring s, jboolean *c) {
	(void) env; if (c) *c = JNI_FALSE; return (const char *) s->data;
}
static void f_ReleaseStringUTFChars (JNIEnv *env, jstring s, const char *p) { (void) env; (void) s; (void) p; }
static jboolean f_IsSameObject (JNIEnv *env, jobject a, jobject b) { (void) env; return a == b; }
static jclass f_FindClass (JNIEnv *env, const char *name) {
	(void) env;
	if (strcmp (name, "java/lang/Integer") != 0) { fprintf (stderr, "FindClass(%s)\n", name); exit (2); }
	return &integer_class;
}
static jmethodID f_GetStaticMethodID (JNIEnv *env, jclass c, const char *n, const char *sig) {
	(void) env; (void) c;
	if (strcmp (n, "valueOf") || strcmp (sig, "(I)Ljava/lang/Integer;")) { fprintf (stderr, "%s%s\n", n, sig); exit (2); }
	return &method;
}
static jmethodID f_GetMethodID (JNIEnv *env, jclass c, const char *n, const char *sig) {
	(void) env; (void) c;
	if (strcmp (n, "intValue") || strcmp (sig, "()I")) { fprintf (stderr, "%s%s\n", n, sig); exit (2); }
	return &method;
}
static jobject f_CallStaticObjectMethod (JNIEnv *env, jclass c, jmethodID m, ...) {
	(void) env; (void) c; (void) m;
	va_list ap;
	va_start (ap, m);
	jint v = va_arg (ap, jint);
	va_end (ap);
	struct _jobject *o = calloc (1, sizeof *o);
	o->kind = OBJ_INTEGER;
	o->value = v;
	++boxes;
	return o;
}
static jint f_CallIntMethod (JNIEnv *env, jobject o, jmethodID m, ...) {
	(void) env; (void) m;
	if (o->kind != OBJ_INTEGER) { fprintf (stderr, "intValue on a non-Integer\n"); exit (2); }
	return o->value;
}

static const struct JNINativeInterface_ table = {
	f_GetArrayLength, f_GetIntArrayElements, f_ReleaseIntArrayElements, f_GetFloatArrayElements,
	f_ReleaseFloatArrayElements, f_GetDirectBufferAddress, f_GetStringUTFChars, f_ReleaseStringUTFChars,
	f_IsSameObject, f_FindClass, f_GetStaticMethodID, f_GetMethodID, f_CallStaticObjectMethod, f_CallIntMethod,
};

static struct _jobject int_array (jint *v, jint n) { struct _jobject o = { OBJ_INT_ARRAY, n, v, 0 }; return o; }
static struct _jobject buffer (void *p) { struct _jobject o = { OBJ_BUFFER, 0, p, 0 }; return o; }
static struct _jobject string (const char *s) { struct _jobject o = { OBJ_STRING, (jint) strlen (s), (void *) s, 0 }; return o; }

/* ---- the natives (TheGPU.java:174-359) ---------------------------------- */
#define NATIVE(ret, name) JNIEXPORT ret JNICALL Java_uk_ac_imperial_lsds_crossbow_device_TheGPU_##name
NATIVE(jint, init) (JNIEnv *, jobject, jintArray, jint, jint, jint, jint, jint);
NATIVE(jint, free) (JNIEnv *, jobject);
NATIVE(jint, setModel) (JNIEnv *, jobject, jint, jint);
NATIVE(jint, setModelVariable) (JNIEnv *, jobject, jint, jint, jintArray, jint);
NATIVE(jint, setModelVariableBuffer) (JNIEnv *, jobject, jint, jint, jobject);
NATIVE(jint, setModelWorkPerClock) (JNIEnv *, jobject, jint);
NATIVE(jint, setUpdateModelType) (JNIEnv *, jobject, jint);
NATIVE(jint, setLearningRateDecayPolicyFixed) (JNIEnv *, jobject, jfloat);
NATIVE(jint, setBaseModelMomentum) (JNIEnv *, jobject, jfloat);
NATIVE(jint, setMomentum) (JNIEnv *, jobject, jfloat, jint);
NATIVE(jint, setWeightDecay) (JNIEnv *, jobject, jfloat);
NATIVE(jint, setEamsgdAlpha) (JNIEnv *, jobject, jfloat);
NATIVE(jint, setModelManager) (JNIEnv *, jobject, jint, jint);
NATIVE(jint, lockAny) (JNIEnv *, jobject);
NATIVE(jint, merge) (JNIEnv *, jobject, jboolean);
NATIVE(jint, synchronise) (JNIEnv *, jobject, jint, jint, jint, jboolean);
NATIVE(jint, unlockAny) (JNIEnv *, jobject);
NATIVE(jint, checkpointModel) (JNIEnv *, jobject, jstring);
NATIVE(jint, overrideModelData) (JNIEnv *, jobject, jstring);
NATIVE(jint, addModel) (JNIEnv *, jobject);
NATIVE(jint, delModel) (JNIEnv *, jobject);
NATIVE(jobject, acquireAccess) (JNIEnv *, jobject, jintArray);
NATIVE(jobject, upgradeAccess) (JNIEnv *, jobject, jobject, jintArray);
#define CALL(name, ...) Java_uk_ac_imperial_lsds_crossbow_device_TheGPU_##name (&env, &self, ##__VA_ARGS__)

extern cbx_context *crossbow_sma_context (void);  /* TheGPU_jni.c */

#define EXPECT(cond)                                                                     \
	do {                                                                                 \
		if (! (cond)) {                                                                  \
			fprintf (stderr, "%s:%d expectation failed: %s\n", __FILE__, __LINE__, #cond); \
			exit (1);                                                                    \
		}                                                                                \
	} while (0)

static void read_floats (const char *path, float *out, size_t n) {
	FILE *f = fopen (path, "rb");
	if (! f) { fprintf (stderr, "missing %s\n", path); exit (1); }
	size_t got = fread (out, sizeof (float), n, f);
	char extra;
	int more = (int) fread (&extra, 1, 1, f);
	fclose (f);
	if (got != n || more) { fprintf (stderr, "%s: %zu floats, %s\n", path, got, more ? "and more" : "short"); exit (1); }
}

static int same_bits (const float *a, const float *b, size_t n) { return memcmp (a, b, n * sizeof (float)) == 0; }

int main (int argc, char **argv) {
	JNIEnv env = &table;
	struct _jobject self = { OBJ_CLASS, 0, NULL, 0 };
	const int G = argc > 1 ? atoi (argv[1]) : 1;
	const int n1 = 40000, n2 = 3331, n = n1 + n2, R = 3, size = R * G;
	const float alpha = 0.1f, momentum = 0.9f;
	EXPECT (G >= 1 && G <= 8);

	/* TheGPU.init: G devices */
	jint devs[8] = { 0 };
	struct _jobject d = int_array (devs, G);
	EXPECT (CALL (init, &d, 2, 2, 2, 0, 0) == 0);

	/* Model.GPURegister (Model.java:338-371): two variables, theModel's values */
	float *z0 = malloc (sizeof (float) * n);
	cbo_fill_normal (z0, (size_t) n, CBO_SEED ^ CBO_BUF_Z, 0.05f, NULL);
	EXPECT (CALL (setModel, 2, 4 * n) == 0);
	jint s1[2] = { n1 / 4, 4 }, s2[1] = { n2 };
	struct _jobject a1 = int_array (s1, 2), a2 = int_array (s2, 1);
	EXPECT (CALL (setModelVariable, 0, 1, &a1, 4 * n1) == 0);
	EXPECT (CALL (setModelVariable, 1, 1, &a2, 4 * n2) == 0);
	struct _jobject b1 = buffer (z0), b2 = buffer (z0 + n1);
	EXPECT (CALL (setModelVariableBuffer, 0, 1, &b1) == 0);
	EXPECT (CALL (setModelVariableBuffer, 1, 1, &b2) == 0);
	EXPECT (CALL (setModelWorkPerClock, 2) == 0);
	EXPECT (CALL (setUpdateModelType, CBX_UPDATE_SMA) == 0);

	/* SolverConf.GPURegister (SolverConf.java:355-409) */
	EXPECT (CALL (setLearningRateDecayPolicyFixed, 0.05f) == 0);
	EXPECT (CALL (setBaseModelMomentum, 0.9f) == 0);
	EXPECT (CALL (setMomentum, momentum, 0) == 0);
	EXPECT (CALL (setWeightDecay, 0.0f) == 0);
	EXPECT (CALL (setEamsgdAlpha, alpha) == 0);

	/* ModelManager (ModelManager.java:87): R replicas per GPU, BSP */
	EXPECT (CALL (setModelManager, R, CBX_SYNC_BSP) == 0);
	cbx_context *ctx = crossbow_sma_context ();
	EXPECT (ctx != NULL && cbx_num_replicas (ctx) == size && cbx_num_devices (ctx) == G);

	/* TaskProcessor (TaskProcessor.java:90-120): reserve a replica per task,
	 * the task runs, the callback handler releases it (callbackhandler.c:154-155). */
	jint clock[1] = { -1 };
	struct _jobject ca = int_array (clock, 1);
	for (int t = 0; t < size; ++t) {
		jobject id = CALL (acquireAccess, &ca);
		EXPECT (id != NULL && id->kind == OBJ_INTEGER && id->value == t && clock[0] == 0);
		clock[0] = -1;
		EXPECT (CALL (upgradeAccess, id, &ca) == id && clock[0] == 0);
		EXPECT (CALL (upgradeAccess, NULL, &ca) == NULL);
		EXPECT (cbx_replica_lock (ctx, id->value) == 0);
		EXPECT (cbx_replica_task_done (ctx, id->value) == 0);
		EXPECT (cbx_replica_release (ctx, id->value) == 0);
		free (id);
	}
	EXPECT (boxes == size);

	/* ResultCollector -> ModelManager.trySynchronise (ModelManager.java:293-353) */
	EXPECT (CALL (lockAny) == size);
	EXPECT (CALL (merge, JNI_FALSE) == 0);  /* first locked replica with updates */
	EXPECT (CALL (synchronise, 0, 1, 0, JNI_FALSE) == 0);
	EXPECT (CALL (unlockAny) == size);

	/* checkpointModel writes dir/000001 in the reference's format */
	char dir[] = "/tmp/cbx_jni_driverXXXXXX";
	EXPECT (mkdtemp (dir) != NULL);
	struct _jobject js = string (dir);
	EXPECT (CALL (checkpointModel, &js) == 0);

	/* The oracle: replicas and theModel start as z0, s_i = 0 (no task
	 * produced a snapshot), last = 0; one SMA step over all replicas of
	 * all G devices (replica i on device i % G). */
	float *z[8], *last[8];
	for (int g = 0; g < G; ++g) {
		z[g] = malloc (sizeof (float) * n);
		last[g] = calloc ((size_t) n, sizeof (float));
		memcpy (z[g], z0, sizeof (float) * n);
	}
	float *s[24], *w[24];
	int locked[24], copy[24];
	for (int i = 0; i < size; ++i) {
		s[i] = calloc ((size_t) n, sizeof (float));
		w[i] = malloc (sizeof (float) * n);
		memcpy (w[i], z0, sizeof (float) * n);
		locked[i] = 1;
		copy[i] = 0;
	}
	float *scratch = malloc (sizeof (float) * (size_t) (G + 1) * (size_t) n);
	EXPECT (cbo_sma_fma (G, size, (size_t) n, alpha, momentum, z, last, s, w, locked, copy, 0, scratch) == 0);

	float *got = malloc (sizeof (float) * n);
	char path[512];
	for (int g = 0; g < G; ++g) {
		/* one device per file set; a selection repeating device 0 names them by position */
		snprintf (path, sizeof path, "%s/000001/gpu-%02d-theModel-data.dat", dir, g);
		read_floats (path, got, (size_t) n);
		EXPECT (same_bits (got, z[g], (size_t) n));
		snprintf (path, sizeof path, "%s/000001/gpu-%02d-theModel-last.dat", dir, g);
		read_floats (path, got, (size_t) n);
		EXPECT (same_bits (got, last[g], (size_t) n));
		EXPECT (same_bits (z[g], z[0], (size_t) n));  /* every device applied the same D */
	}
	for (int i = 0; i < size; ++i) {
		snprintf (path, sizeof path, "%s/000001/gpu-%02d-replica-%03d-data.dat", dir, i % G, i);
		read_floats (path, got, (size_t) n);
		EXPECT (same_bits (got, w[i], (size_t) n));
	}
	EXPECT (! same_bits (z[0], z0, (size_t) n));  /* the step did move z */

	/* Another step, then overrideModelData from 000001 and a new checkpoint:
	 * 000002 must hold 000001's values again. */
	EXPECT (CALL (lockAny) == size);
	EXPECT (CALL (synchronise, 0, 2, 0, JNI_FALSE) == 0);
	EXPECT (CALL (unlockAny) == size);
	char version[512];
	snprintf (version, sizeof version, "%s/000001", dir);
	struct _jobject jv = string (version);
	EXPECT (CALL (overrideModelData, &jv) == 0);
	EXPECT (CALL (overrideModelData, NULL) == 0);  /* GPU.c:1169: a null directory is a no-op */
	EXPECT (CALL (checkpointModel, &js) == 0);
	for (int g = 0; g < G; ++g) {
		snprintf (path, sizeof path, "%s/000002/gpu-%02d-theModel-data.dat", dir, g);
		read_floats (path, got, (size_t) n);
		EXPECT (same_bits (got, z[g], (size_t) n));
	}

	/* Autotune's addModel / delModel (GPU.c:1178-1199) */
	EXPECT (CALL (lockAny) == size);
	EXPECT (CALL (addModel) == 0);  /* one more replica per device */
	EXPECT (cbx_num_replicas (ctx) == size + G);
	EXPECT (CALL (unlockAny) == size + G);
	EXPECT (CALL (lockAny) == size + G);
	EXPECT (CALL (delModel) == 0);
	EXPECT (cbx_num_replicas (ctx) == size);
	EXPECT (CALL (unlockAny) == size);

	EXPECT (CALL (free) == 0);
	EXPECT (crossbow_sma_context () == NULL);
	printf ("jni_driver: ok (G=%d)\n", G);
	fflush (stdout);
	_exit (0);
}

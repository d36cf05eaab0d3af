/* Minimal stand-in for a JDK's jni.h, used ONLY by tests/test_abi.py to
 * compile-check crossbow_amd/csrc/jni/TheGPU_jni.c (gcc -fsyntax-only) in an
 * image without a JDK.  Declares just the types, macros and JNIEnv function
 * slots the shim uses, with the JNI specification's signatures.  Never
 * linked into anything. */
#ifndef CBX_TEST_JNI_STUB_H
#define CBX_TEST_JNI_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jintArray;
typedef jobject jfloatArray;
typedef jobject jstring;
typedef jobject jclass;
typedef struct _jmethodID *jmethodID;
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
	jsize (*GetArrayLength) (JNIEnv *, jobject);
	jint *(*GetIntArrayElements) (JNIEnv *, jintArray, jboolean *);
	void (*ReleaseIntArrayElements) (JNIEnv *, jintArray, jint *, jint);
	jfloat *(*GetFloatArrayElements) (JNIEnv *, jfloatArray, jboolean *);
	void (*ReleaseFloatArrayElements) (JNIEnv *, jfloatArray, jfloat *, jint);
	void *(*GetDirectBufferAddress) (JNIEnv *, jobject);
	const char *(*GetStringUTFChars) (JNIEnv *, jstring, jboolean *);
	void (*ReleaseStringUTFChars) (JNIEnv *, jstring, const char *);
	jboolean (*IsSameObject) (JNIEnv *, jobject, jobject);
	jclass (*FindClass) (JNIEnv *, const char *);
	jmethodID (*GetStaticMethodID) (JNIEnv *, jclass, const char *, const char *);
	jmethodID (*GetMethodID) (JNIEnv *, jclass, const char *, const char *);
	jobject (*CallStaticObjectMethod) (JNIEnv *, jclass, jmethodID, ...);
	jint (*CallIntMethod) (JNIEnv *, jobject, jmethodID, ...);
};
#endif

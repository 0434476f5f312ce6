/* Minimal jni.h for a syntax / type check of integration/jni/dukehip_jni.c in an image
 * without a JDK (tests/test_jni_glue.py).  Hand-written from the JNI specification: only the
 * types and the JNIEnv functions the glue uses, with their specified C signatures.  It is a
 * checker, never linked or shipped. */
#ifndef DK_TEST_JNI_STUB_H
#define DK_TEST_JNI_STUB_H
#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jcharArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*Throw)(JNIEnv*, jthrowable);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jboolean (*ExceptionCheck)(JNIEnv*);
  void (*ExceptionClear)(JNIEnv*);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
  jmethodID (*GetMethodID)(JNIEnv*, jclass, const char*, const char*);
  jobject (*NewObject)(JNIEnv*, jclass, jmethodID, ...);
  jstring (*NewString)(JNIEnv*, const jchar*, jsize);
  jsize (*GetStringLength)(JNIEnv*, jstring);
  const jchar* (*GetStringChars)(JNIEnv*, jstring, jboolean*);
  void (*ReleaseStringChars)(JNIEnv*, jstring, const jchar*);
  void (*GetStringRegion)(JNIEnv*, jstring, jsize, jsize, jchar*);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  const char* (*GetStringUTFChars)(JNIEnv*, jstring, jboolean*);
  void (*ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jobjectArray (*NewObjectArray)(JNIEnv*, jsize, jclass, jobject);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jintArray (*NewIntArray)(JNIEnv*, jsize);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  jdoubleArray (*NewDoubleArray)(JNIEnv*, jsize);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  jchar* (*GetCharArrayElements)(JNIEnv*, jcharArray, jboolean*);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
  jdouble* (*GetDoubleArrayElements)(JNIEnv*, jdoubleArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  void (*ReleaseCharArrayElements)(JNIEnv*, jcharArray, jchar*, jint);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
  void (*ReleaseDoubleArrayElements)(JNIEnv*, jdoubleArray, jdouble*, jint);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void (*SetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*);
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
};

#endif

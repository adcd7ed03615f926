/* Minimal JNI declarations for type-checking jni/clonos_jni.c in this container (no JDK
 * here).  TEST INFRASTRUCTURE: only the types and JNIEnv functions the shim uses, with
 * the signatures of the JNI specification; a real build uses $JAVA_HOME/include/jni.h. */
#ifndef CLONOS_TEST_JNI_STUB_H
#define CLONOS_TEST_JNI_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int16_t jshort;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef void* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jbyteArray;
typedef jarray jobjectArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
};
#endif

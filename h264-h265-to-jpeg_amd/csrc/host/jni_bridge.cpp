// JNI export, ABI-identical to the reference's
// Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode
// (/root/reference/src/jni/com_autonavi_socol_occtiltedserver_service_H265DecodeService.cpp:10-30,
// signature (Ljava/lang/String;Ljava/lang/String;)Z).  No JDK in this image:
// the JNIEnv function table is addressed by its standard indices
// (GetStringUTFChars = 169, ReleaseStringUTFChars = 170 in JNINativeInterface_).
// Unlike the reference, the UTF chars are released (the reference leaks
// both strings on every call, :13-14).
#include "IDecoder.h"

extern "C" {
typedef unsigned char jboolean;
typedef void* jobject;
typedef jobject jclass;
typedef jobject jstring;
struct JNIEnvOpaque;
typedef JNIEnvOpaque JNIEnv;

typedef const char* (*GetUTF)(JNIEnv*, jstring, jboolean*);
typedef void (*ReleaseUTF)(JNIEnv*, jstring, const char*);

__attribute__((visibility("default"))) jboolean
Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode(JNIEnv* env, jclass, jstring inputPath,
                                                                       jstring outputPath) {
    void* const* table = *reinterpret_cast<void* const* const*>(env);
    GetUTF get = reinterpret_cast<GetUTF>(table[169]);
    ReleaseUTF rel = reinterpret_cast<ReleaseUTF>(table[170]);
    const char* input = get(env, inputPath, nullptr);
    const char* output = get(env, outputPath, nullptr);
    bool ok = false;
    auto decoder = IDecoder::getInstance();
    if (decoder && input && output) ok = decoder->H265ToJpeg(input, output);
    if (input) rel(env, inputPath, input);
    if (output) rel(env, outputPath, output);
    return ok ? 1 : 0;
}
}

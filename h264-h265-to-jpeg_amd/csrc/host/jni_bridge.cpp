// JNI export, ABI-identical to the reference's
// Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode
// (/root/reference/src/jni/com_autonavi_socol_occtiltedserver_service_H265DecodeService.cpp:10-30,
// signature (Ljava/lang/String;Ljava/lang/String;)Z).  No JDK in this image:
// the JNIEnv function table is addressed by its standard indices
// (GetStringUTFChars = 169, ReleaseStringUTFChars = 170 in JNINativeInterface_).
// Unlike the reference, the UTF chars are released (the reference leaks
// both strings on every call, :13-14).
#include <cstdint>
#include <vector>

#include "IDecoder.h"
#include "h2j.h"

extern "C" {
typedef unsigned char jboolean;
typedef void* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jbooleanArray;
typedef jarray jobjectArray;
typedef int32_t jsize;
typedef signed char jbyte;
struct JNIEnvOpaque;
typedef JNIEnvOpaque JNIEnv;

typedef const char* (*GetUTF)(JNIEnv*, jstring, jboolean*);
typedef void (*ReleaseUTF)(JNIEnv*, jstring, const char*);
// further JNINativeInterface_ slots used by the byte[] / batch variants
typedef jsize (*GetArrayLength)(JNIEnv*, jarray);                                            // 171
typedef jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);                      // 173
typedef jbooleanArray (*NewBooleanArray)(JNIEnv*, jsize);                                    // 175
typedef jbyteArray (*NewByteArray)(JNIEnv*, jsize);                                          // 176
typedef void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);               // 200
typedef void (*SetBooleanArrayRegion)(JNIEnv*, jbooleanArray, jsize, jsize, const jboolean*);  // 207
typedef void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);         // 208

static void* const* jni_table(JNIEnv* env) { return *reinterpret_cast<void* const* const*>(env); }

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

// In-memory variant: `static native byte[] decodeBytes(byte[] input)` on the same
// Java class -> the JPEG bytes, or null on failure (the LOG line says why).
__attribute__((visibility("default"))) jbyteArray
Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBytes(JNIEnv* env, jclass, jbyteArray input) {
    void* const* t = jni_table(env);
    if (!input) return nullptr;
    const jsize n = reinterpret_cast<GetArrayLength>(t[171])(env, input);
    if (n <= 0) return nullptr;
    std::vector<uint8_t> data(static_cast<size_t>(n));
    reinterpret_cast<GetByteArrayRegion>(t[200])(env, input, 0, n, reinterpret_cast<jbyte*>(data.data()));
    uint8_t* jpeg = nullptr;
    size_t len = 0;
    if (h2j_h265_to_jpeg_mem(data.data(), data.size(), &jpeg, &len) != 0) return nullptr;
    jbyteArray out = reinterpret_cast<NewByteArray>(t[176])(env, static_cast<jsize>(len));
    if (out) reinterpret_cast<SetByteArrayRegion>(t[208])(env, out, 0, static_cast<jsize>(len), reinterpret_cast<const jbyte*>(jpeg));
    h2j_free(jpeg);
    return out;
}

// Batch variant: `static native boolean[] decodeBatch(String[] inputs, String[] outputs)`, one
// GPU batch for all pairs; element i is what decode(inputs[i], outputs[i]) would return.
__attribute__((visibility("default"))) jbooleanArray
Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBatch(JNIEnv* env, jclass, jobjectArray inputs,
                                                                            jobjectArray outputs) {
    void* const* t = jni_table(env);
    if (!inputs || !outputs) return nullptr;
    GetArrayLength len = reinterpret_cast<GetArrayLength>(t[171]);
    const jsize n = len(env, inputs);
    if (n < 0 || len(env, outputs) != n) return nullptr;
    GetObjectArrayElement elem = reinterpret_cast<GetObjectArrayElement>(t[173]);
    GetUTF get = reinterpret_cast<GetUTF>(t[169]);
    ReleaseUTF rel = reinterpret_cast<ReleaseUTF>(t[170]);
    std::vector<jstring> js_in(n), js_out(n);
    std::vector<const char*> in(n), out(n);
    for (jsize i = 0; i < n; i++) {
        js_in[i] = elem(env, inputs, i);
        js_out[i] = elem(env, outputs, i);
        in[i] = js_in[i] ? get(env, js_in[i], nullptr) : nullptr;
        out[i] = js_out[i] ? get(env, js_out[i], nullptr) : nullptr;
    }
    std::vector<int> ok(n, 0);
    if (n > 0) h2j_h265_to_jpeg_batch(in.data(), out.data(), n, ok.data());
    for (jsize i = 0; i < n; i++) {
        if (in[i]) rel(env, js_in[i], in[i]);
        if (out[i]) rel(env, js_out[i], out[i]);
    }
    jbooleanArray res = reinterpret_cast<NewBooleanArray>(t[175])(env, n);
    if (res && n > 0) {
        std::vector<jboolean> b(n);
        for (jsize i = 0; i < n; i++) b[i] = ok[i] ? 1 : 0;
        reinterpret_cast<SetBooleanArrayRegion>(t[207])(env, res, 0, n, b.data());
    }
    return res;
}
}

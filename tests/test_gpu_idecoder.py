"""The C++ drop-in surface: a program written against the reference's
IDecoder.h (README.md:38-54 usage) links libH265ToJpeg.so and transcodes."""
import os
import subprocess

import pytest

from conftest import golden, read

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-h265-to-jpeg_amd")

DRIVER = r'''
#include "IDecoder.h"
#include <cstdio>
int main(int argc, char** argv) {
    auto decoder = IDecoder::getInstance();
    if (!decoder) return 3;
    bool ok = decoder->H265ToJpeg(argv[1], argv[2]);
    bool bad = IDecoder::getInstance()->H265ToJpeg("", argv[2]);
    return ok && !bad ? 0 : 1;
}
'''


def test_idecoder_cpp_driver(tmp_path):
    src = tmp_path / "drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.check_call(["g++", "-std=c++11", "-O1", str(src), "-I", os.path.join(ROOT, "include"), "-L", PKG,
                           "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    out = tmp_path / "out.jpg"
    r = subprocess.run([str(exe), golden("img01.h265"), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import oracle_py as O
    assert out.read_bytes() == O.transcode(read(golden("img01.h265")))


def test_python_h265_to_jpeg(tmp_path):
    import h2j
    out = tmp_path / "o.jpg"
    assert h2j.h265_to_jpeg(golden("img01.h265"), str(out))
    assert not h2j.h265_to_jpeg(str(tmp_path / "missing.h265"), str(out))


CONCURRENT = r'''
#include "IDecoder.h"
#include <string>
#include <thread>
#include <vector>
// the reference's instances are independent (no global state, src/Decoder.cpp:10-12,45-52);
// here concurrent calls from many threads are batched onto the shared engine
int main(int argc, char** argv) {
    const int n = 12;
    std::vector<int> ok(n, 0);
    std::vector<std::thread> th;
    for (int i = 0; i < n; i++)
        th.emplace_back([&, i]() {
            const char* in = argv[1 + (i % 2)];
            std::string out = std::string(argv[3]) + "/o" + std::to_string(i) + ".jpg";
            ok[i] = IDecoder::getInstance()->H265ToJpeg(in, out.c_str()) ? 1 : 0;
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; i++)
        if (!ok[i]) return 1;
    return 0;
}
'''


def test_idecoder_concurrent_calls_are_batched_and_exact(tmp_path):
    src = tmp_path / "conc.cpp"
    src.write_text(CONCURRENT)
    exe = tmp_path / "conc"
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-pthread", str(src), "-I", os.path.join(ROOT, "include"),
                           "-L", PKG, "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    r = subprocess.run([str(exe), golden("img01.h265"), golden("img01.h264"), str(tmp_path)], capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    import oracle_py as O
    want = [O.transcode(read(golden("img01.h265"))), O.transcode(read(golden("img01.h264")))]
    for i in range(12):
        assert (tmp_path / f"o{i}.jpg").read_bytes() == want[i % 2], i


JNI_DRIVER = r'''
/* Drives the JNI export the way a JVM would, with a minimal JNIEnv whose
 * function table holds GetStringUTFChars (169) and ReleaseStringUTFChars (170)
 * (JNINativeInterface_ order); a jstring is represented by a C string. */
#include <stdio.h>
#include <string.h>
typedef unsigned char jboolean;
typedef void* jobject;
static int released = 0;
static const char* get_utf(void* env, jobject s, jboolean* copy) { (void)env; if (copy) *copy = 0; return (const char*)s; }
static void rel_utf(void* env, jobject s, const char* c) { (void)env; (void)s; (void)c; released++; }
extern jboolean Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode(void*, jobject, jobject, jobject);
int main(int argc, char** argv) {
    void* table[232];
    memset(table, 0, sizeof(table));
    table[169] = (void*)get_utf;
    table[170] = (void*)rel_utf;
    void** env = table;  /* JNIEnv* points at a struct whose first member is the table pointer */
    jboolean ok = Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode(&env, 0, argv[1], argv[2]);
    jboolean bad = Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decode(&env, 0, (char*)"", argv[2]);
    printf("ok=%d bad=%d released=%d\n", ok, bad, released);
    return ok == 1 && bad == 0 && released == 4 ? 0 : 1;
}
'''


def test_jni_export_with_stub_env(tmp_path):
    src = tmp_path / "jni.c"
    src.write_text(JNI_DRIVER)
    exe = tmp_path / "jni"
    subprocess.check_call(["gcc", "-O1", str(src), "-L", PKG, "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    out = tmp_path / "jni.jpg"
    r = subprocess.run([str(exe), golden("img01.h265"), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    import oracle_py as O
    assert out.read_bytes() == O.transcode(read(golden("img01.h265")))

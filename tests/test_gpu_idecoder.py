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


MEM_BATCH_DRIVER = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h2j.h"
/* argv: in265 in264 outdir -> mem transcode of in265 to outdir/m.jpg, batch of
 * (in265, in264, missing, "") to outdir/b0..b3.jpg */
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    rewind(f);
    unsigned char* d = (unsigned char*)malloc(n);
    if (fread(d, 1, n, f) != (size_t)n) return 5;
    fclose(f);
    unsigned char* jpeg = 0;
    size_t len = 0;
    if (h2j_h265_to_jpeg_mem(d, n, &jpeg, &len) != 0 || !jpeg) return 2;
    char p[4096];
    snprintf(p, sizeof p, "%s/m.jpg", argv[3]);
    f = fopen(p, "wb");
    fwrite(jpeg, 1, len, f);
    fclose(f);
    h2j_free(jpeg);
    if (h2j_h265_to_jpeg_mem(d, 16, &jpeg, &len) == 0 || jpeg) return 3; /* truncated input fails */
    const char* in[4] = {argv[1], argv[2], "/nonexistent/x.h265", ""};
    char outs[4][4096];
    const char* out[4];
    for (int i = 0; i < 4; i++) { snprintf(outs[i], sizeof outs[i], "%s/b%d.jpg", argv[3], i); out[i] = outs[i]; }
    int ok[4] = {9, 9, 9, 9};
    int good = h2j_h265_to_jpeg_batch(in, out, 4, ok);
    printf("good=%d ok=%d%d%d%d\n", good, ok[0], ok[1], ok[2], ok[3]);
    return good == 2 && ok[0] == 1 && ok[1] == 1 && ok[2] == 0 && ok[3] == 0 ? 0 : 4;
}
'''


def test_mem_and_batch_entry_points(tmp_path):
    src = tmp_path / "mb.c"
    src.write_text(MEM_BATCH_DRIVER)
    exe = tmp_path / "mb"
    subprocess.check_call(["gcc", "-O1", str(src), "-I", os.path.join(ROOT, "include"), "-L", PKG, "-lH265ToJpeg",
                           f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    r = subprocess.run([str(exe), golden("img01.h265"), golden("img01.h264"), str(tmp_path)], capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    import oracle_py as O
    w265 = O.transcode(read(golden("img01.h265")))
    assert (tmp_path / "m.jpg").read_bytes() == w265
    assert (tmp_path / "b0.jpg").read_bytes() == w265
    assert (tmp_path / "b1.jpg").read_bytes() == O.transcode(read(golden("img01.h264")))
    assert not (tmp_path / "b2.jpg").exists() and not (tmp_path / "b3.jpg").exists()


JNI_ARRAYS_DRIVER = r'''
/* decodeBytes / decodeBatch driven through a stub JNIEnv: a jbyteArray is a
 * {len, bytes} struct, a String[] a {len, char**} struct, a boolean[] a
 * {len, bytes} struct (JNINativeInterface_ slots 169-176, 200, 207, 208). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef unsigned char jboolean;
typedef struct { int len; unsigned char* b; } Arr;
typedef struct { int len; const char** s; } SArr;
static const char* get_utf(void* e, void* s, jboolean* c) { (void)e; if (c) *c = 0; return (const char*)s; }
static void rel_utf(void* e, void* s, const char* c) { (void)e; (void)s; (void)c; }
static int arr_len(void* e, void* a) { (void)e; return ((Arr*)a)->len; }
static void* obj_elem(void* e, void* a, int i) { (void)e; return (void*)((SArr*)a)->s[i]; }
static void* new_arr(void* e, int n) { (void)e; Arr* a = malloc(sizeof(Arr)); a->len = n; a->b = calloc(n + 1, 1); return a; }
static void get_region(void* e, void* a, int s, int n, signed char* d) { (void)e; memcpy(d, ((Arr*)a)->b + s, n); }
static void set_region(void* e, void* a, int s, int n, const void* d) { (void)e; memcpy(((Arr*)a)->b + s, d, n); }
extern void* Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBytes(void*, void*, void*);
extern void* Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBatch(void*, void*, void*, void*);
int main(int argc, char** argv) {
    void* table[232];
    memset(table, 0, sizeof(table));
    table[169] = (void*)get_utf; table[170] = (void*)rel_utf; table[171] = (void*)arr_len;
    table[173] = (void*)obj_elem; table[175] = (void*)new_arr; table[176] = (void*)new_arr;
    table[200] = (void*)get_region; table[207] = (void*)set_region; table[208] = (void*)set_region;
    void** env = table;
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    Arr in; in.len = (int)ftell(f); rewind(f); in.b = malloc(in.len);
    if (fread(in.b, 1, in.len, f) != (size_t)in.len) return 5;
    fclose(f);
    Arr* out = Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBytes(&env, 0, &in);
    if (!out) return 2;
    f = fopen(argv[3], "wb"); fwrite(out->b, 1, out->len, f); fclose(f);
    const char* ins[2] = {argv[1], "/nonexistent.h265"};
    const char* outs[2] = {argv[4], argv[5]};
    SArr si = {2, ins}, so = {2, outs};
    Arr* ok = Java_com_autonavi_socol_occtiltedserver_service_H265DecodeService_decodeBatch(&env, 0, &si, &so);
    if (!ok || ok->len != 2) return 3;
    printf("ok=%d%d\n", ok->b[0], ok->b[1]);
    return ok->b[0] == 1 && ok->b[1] == 0 ? 0 : 4;
}
'''


def test_jni_bytes_and_batch_with_stub_env(tmp_path):
    src = tmp_path / "jarr.c"
    src.write_text(JNI_ARRAYS_DRIVER)
    exe = tmp_path / "jarr"
    subprocess.check_call(["gcc", "-O1", str(src), "-L", PKG, "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    o1, o2, o3 = tmp_path / "bytes.jpg", tmp_path / "batch0.jpg", tmp_path / "batch1.jpg"
    r = subprocess.run([str(exe), golden("img01.h264"), "unused", str(o1), str(o2), str(o3)], capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    import oracle_py as O
    want = O.transcode(read(golden("img01.h264")))
    assert o1.read_bytes() == want and o2.read_bytes() == want and not o3.exists()


MULTI_ENGINE_DRIVER = r'''
#include <stdio.h>
#include <stdlib.h>
#include "h2j.h"
/* argv: outdir in1 in2 ... -> h2j_h265_to_jpeg_batch over all inputs into outdir/o<i>.jpg */
int main(int argc, char** argv) {
    int n = argc - 2;
    const char** in = (const char**)calloc(n, sizeof(char*));
    const char** out = (const char**)calloc(n, sizeof(char*));
    int* ok = (int*)calloc(n, sizeof(int));
    for (int i = 0; i < n; i++) {
        char* p = (char*)malloc(4096);
        snprintf(p, 4096, "%s/o%d.jpg", argv[1], i);
        in[i] = argv[2 + i];
        out[i] = p;
    }
    int good = h2j_h265_to_jpeg_batch(in, out, n, ok);
    printf("good=%d\n", good);
    return 0;
}
'''


@pytest.mark.parametrize("engines", ["2", "3"])
def test_facade_splits_batches_over_engines(tmp_path, engines):
    """The IDecoder / batch facade runs one engine per GPU (H2J_ENGINES overrides the count, so
    a one-GPU box exercises the split): a batch is LPT-split over the idle engines and every
    JPEG stays byte-exact; a malformed input fails alone, its LOG line carries its own message."""
    import glob
    import oracle_py as O
    src = tmp_path / "me.c"
    src.write_text(MULTI_ENGINE_DRIVER)
    exe = tmp_path / "me"
    subprocess.check_call(["gcc", "-O1", str(src), "-I", os.path.join(ROOT, "include"), "-L", PKG, "-lH265ToJpeg",
                           f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    ins = sorted(glob.glob(golden("hevc/*.h265")))[:10] + sorted(glob.glob(golden("h264/*.h264")))[:10]
    bad = golden("malformed/m_avc_firstmb_oob.h264")
    ins.insert(7, bad)
    env = dict(os.environ, H2J_ENGINES=engines)
    r = subprocess.run([str(exe), str(tmp_path)] + ins, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert f"good={len(ins) - 1}" in r.stdout
    assert "first_mb_in_slice outside the picture" in r.stdout
    for i, p in enumerate(ins):
        if p == bad:
            assert not (tmp_path / f"o{i}.jpg").exists()
        else:
            assert (tmp_path / f"o{i}.jpg").read_bytes() == O.transcode(read(p)), p


def test_concurrent_idecoder_calls_over_two_engines(tmp_path):
    src = tmp_path / "conc.cpp"
    src.write_text(CONCURRENT)
    exe = tmp_path / "conc"
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-pthread", str(src), "-I", os.path.join(ROOT, "include"),
                           "-L", PKG, "-lH265ToJpeg", f"-Wl,-rpath,{PKG}", "-o", str(exe)])
    env = dict(os.environ, H2J_ENGINES="2")
    r = subprocess.run([str(exe), golden("img01.h265"), golden("img01.h264"), str(tmp_path)], capture_output=True,
                       text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    import oracle_py as O
    want = [O.transcode(read(golden("img01.h265"))), O.transcode(read(golden("img01.h264")))]
    for i in range(12):
        assert (tmp_path / f"o{i}.jpg").read_bytes() == want[i % 2], i


def test_engine_host_placement_reported(engine):
    info = engine.host_info()
    assert info["threads"] >= 1
    assert info["pinned_cpus"] == 0 or info["pinned_cpus"] >= 1

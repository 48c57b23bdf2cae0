"""Kernel-source handling: name extraction (reference regex,
ClNumberCruncher.cs:218-228), hidden-offset rewrite, OpenCL-C dialect and
hiprtc compilation for gfx950 (cross-compiles without a GPU)."""
import pytest

from cekirdekler_amd import cek


def test_parse_names_and_arity():
    src = """
    // __global__ void commented(float* a)
    extern "C" __global__ void a1(float* x, const float* __restrict__ y) {}
    __global__ __launch_bounds__(256) void b2() {}
    __global__ void c3(int* a, int* b, int* c) { }
    template <int N> __global__ void templ(float* p) {}
    """
    ks = [(k.name, k.arity) for k in cek.parse_kernels(src)]
    assert ks == [("a1", 2), ("b2", 0), ("c3", 3)]


def test_gpu_rewrite_appends_hidden_args():
    out = cek.gpu_rewrite("__global__ void k(float* x) { x[get_global_id(0)] = 1; }")
    assert 'extern "C" __global__ void k(float* x, long long __cek_off, long long __cek_gsize)' in out
    out0 = cek.gpu_rewrite("__global__ void k() { }")
    assert "void k(long long __cek_off, long long __cek_gsize)" in out0


def test_opencl_dialect_translation():
    src = """
    __kernel void hello(__global float* a, __global const float* b) {
        __local float s[64];
        int i = get_global_id(0);
        s[get_local_id(0)] = b[i];
        barrier(CLK_LOCAL_MEM_FENCE);
        a[i] = s[get_local_id(0)] * 2.0f;
    }"""
    assert cek.is_opencl_dialect(src)
    ks = cek.parse_kernels(src)
    assert [(k.name, k.arity) for k in ks] == [("hello", 2)]
    out = cek.gpu_rewrite(src)
    assert "__shared__ float s[64]" in out and "__syncthreads()" in out


@pytest.mark.parametrize("src", [
    "__global__ void k(float* x) { x[get_global_id(0)] *= 2.0f; }",
    "__kernel void k(__global float* x) { x[get_global_id(0)] *= 2.0f; }",
])
def test_hiprtc_compiles_for_gfx950(src):
    ok, code, log = cek.compile_gpu(src, [], "gfx950")
    assert ok, log
    assert code[:4] == b"\x7fELF"


def test_hiprtc_reports_errors():
    ok, code, log = cek.compile_gpu("__global__ void k(float* x) { x[0] = undefined_symbol; }", [], "gfx950")
    assert not ok
    assert "undefined_symbol" in log


DYN_SRC = r"""
__cek_child__ void fill(long long id, long long param, float* x) {
  x[param + id] += 1.0f;
  if (id == 0 && param == 0) cek_enqueue(fill2, 64, 128);
}
__cek_child__ void fill2(long long id, long long param, float* x) { x[param + id] += 10.0f; }
__global__ void parent(float* x) {
  long long i = get_global_id(0);
  if (i == 0) cek_enqueue(fill, 128, 0);
  x[i] += 100.0f;
}
"""


def test_device_enqueue_rewrite_and_compile():
    """cek_enqueue (the OpenCL 2.0 enqueue_kernel replacement): children get
    the queue + level, the parent gets a generated dispatcher, and the whole
    program cross-compiles for gfx950."""
    out = cek.gpu_rewrite(DYN_SRC)
    assert "__cek_dispatch_parent(float* x, long long __cek_off, long long __cek_gsize, void* __cek_q, int __cek_level)" in out
    assert "void fill(long long id, long long param, float* x, void* __cek_q, int __cek_level)" in out
    assert "case 1: fill2(i, rec.param, x, __cek_q, __cek_level)" in out
    ok, code, log = cek.compile_gpu(DYN_SRC, [], "gfx950")
    assert ok, log
    # plain sources are untouched by the dynamic path
    assert "__cek_dispatch" not in cek.gpu_rewrite("__global__ void k(float* x) { x[0] = 1; }")

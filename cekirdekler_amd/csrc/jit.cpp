#include "jit.h"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <regex>
#include <set>
#include <sstream>

namespace cek {

// ---------------------------------------------------------------- helpers --

std::string hash_hex(const std::string& s) {
  uint64_t h1 = 1469598103934665603ull, h2 = 0x9e3779b97f4a7c15ull;
  for (unsigned char c : s) {
    h1 = (h1 ^ c) * 1099511628211ull;
    h2 = (h2 ^ c) * 0x100000001b3ull + 0x632be59bd9b4e019ull;
  }
  char buf[40];
  snprintf(buf, sizeof(buf), "%016llx%016llx", (unsigned long long)h1, (unsigned long long)h2);
  return buf;
}

static void mkdirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    mkdir(cur.c_str(), 0755);
  }
}

std::string cache_dir() {
  const char* e = getenv("CEK_CACHE_DIR");
  std::string d;
  if (e && *e) {
    d = e;
  } else {
    const char* home = getenv("HOME");
    d = std::string(home && *home ? home : "/tmp") + "/.cache/cekirdekler_amd";
  }
  mkdirs(d);
  return d;
}

static bool read_file(const std::string& p, std::string& out) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  std::ostringstream os;
  os << f.rdbuf();
  out = os.str();
  return true;
}

static void write_file_atomic(const std::string& p, const std::string& data) {
  std::string tmp = p + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    f.write(data.data(), static_cast<std::streamsize>(data.size()));
  }
  rename(tmp.c_str(), p.c_str());
}

// Replace comments with spaces (keeps offsets stable); string literals kept.
static std::string strip_comments(const std::string& s) {
  std::string o = s;
  size_t i = 0, n = s.size();
  while (i < n) {
    if (s[i] == '"' || s[i] == '\'') {
      char q = s[i++];
      while (i < n && s[i] != q) {
        if (s[i] == '\\') ++i;
        ++i;
      }
      ++i;
    } else if (i + 1 < n && s[i] == '/' && s[i + 1] == '/') {
      while (i < n && s[i] != '\n') o[i++] = ' ';
    } else if (i + 1 < n && s[i] == '/' && s[i + 1] == '*') {
      o[i] = o[i + 1] = ' ';
      i += 2;
      while (i + 1 < n && !(s[i] == '*' && s[i + 1] == '/')) {
        if (s[i] != '\n') o[i] = ' ';
        ++i;
      }
      if (i + 1 < n) o[i] = o[i + 1] = ' ';
      i += 2;
    } else {
      ++i;
    }
  }
  return o;
}

bool is_opencl_dialect(const std::string& src) {
  static const std::regex re(R"((^|[^\w])(__kernel|kernel)\s+void\s)");
  return std::regex_search(strip_comments(src), re);
}

static std::string regex_replace_all(const std::string& s, const std::string& pat,
                                     const std::string& rep) {
  return std::regex_replace(s, std::regex(pat), rep);
}

// OpenCL-C → HIP C++ (best effort; the reference's kernels are OpenCL C).
static std::string translate_opencl(const std::string& src) {
  std::string s = strip_comments(src);
  s = regex_replace_all(s, R"((^|[^\w])(__kernel|kernel)(\s+void\s))", "$1__global__$3");
  s = regex_replace_all(s, R"((^|[^\w])__global(?![\w]))", "$1");
  s = regex_replace_all(s, R"((^|[^\w])global(\s+[\w]))", "$1$2");
  s = regex_replace_all(s, R"((^|[^\w])(__local|local)(\s+))", "$1__shared__$3");
  s = regex_replace_all(s, R"((^|[^\w])(__constant|constant)(\s+))", "$1const$3");
  s = regex_replace_all(s, R"((^|[^\w])(__private|private)(\s+))", "$1$3");
  s = regex_replace_all(s, R"(barrier\s*\([^)]*\))", "__syncthreads()");
  s = regex_replace_all(s, R"(mem_fence\s*\([^)]*\))", "__threadfence()");
  return "#define CEK_OPENCL_DIALECT 1\n" + s;
}

static size_t match_paren(const std::string& s, size_t open) {
  int depth = 0;
  for (size_t i = open; i < s.size(); ++i) {
    if (s[i] == '(') ++depth;
    else if (s[i] == ')') {
      if (--depth == 0) return i;
    }
  }
  return std::string::npos;
}

static int count_params(const std::string& inside) {
  std::string t;
  for (char c : inside)
    if (!isspace(static_cast<unsigned char>(c))) t += c;
  if (t.empty() || t == "void") return 0;
  int depth = 0, n = 1;
  for (char c : inside) {
    if (c == '(' || c == '<' || c == '[') ++depth;
    else if (c == ')' || c == '>' || c == ']') --depth;
    else if (c == ',' && depth == 0) ++n;
  }
  return n;
}

struct KernelSite {
  size_t global_pos;   // position of "__global__"
  bool has_extern_c;
  size_t open, close;  // parameter parens
  KernelSig sig;
};

static std::vector<KernelSite> find_sites(const std::string& s) {
  static const std::regex re(
      R"((extern\s+"C"\s+)?__global__\s+(__launch_bounds__\s*\([^)]*\)\s*)?void\s+(__launch_bounds__\s*\([^)]*\)\s*)?([A-Za-z_]\w*)\s*\()");
  std::vector<KernelSite> out;
  for (auto it = std::sregex_iterator(s.begin(), s.end(), re); it != std::sregex_iterator(); ++it) {
    const auto& m = *it;
    // Skip template kernels (cannot be extern "C").
    size_t start = static_cast<size_t>(m.position(0));
    size_t back = start;
    while (back > 0 && isspace(static_cast<unsigned char>(s[back - 1]))) --back;
    if (back > 0 && s[back - 1] == '>') continue;
    KernelSite k;
    k.has_extern_c = m[1].matched;
    k.global_pos = k.has_extern_c ? static_cast<size_t>(m.position(1)) : start;
    k.open = start + static_cast<size_t>(m.length(0)) - 1;
    k.close = match_paren(s, k.open);
    if (k.close == std::string::npos) continue;
    k.sig.name = m[4].str();
    k.sig.arity = count_params(s.substr(k.open + 1, k.close - k.open - 1));
    out.push_back(k);
  }
  return out;
}

std::vector<KernelSig> parse_kernels(const std::string& src) {
  std::string s = is_opencl_dialect(src) ? translate_opencl(src) : strip_comments(src);
  std::vector<KernelSig> out;
  std::set<std::string> seen;
  for (auto& k : find_sites(s)) {
    if (seen.insert(k.sig.name).second) out.push_back(k.sig);
  }
  return out;
}

// ------------------------------------------------------------- preludes --

static const char* kGpuPrelude = R"CEK(
// ---- cekirdekler_amd GPU prelude (gfx950) ----
#define CEK_GPU 1
#define get_global_id(d) ((d) == 0 ? ((long long)blockIdx.x * (long long)blockDim.x + (long long)threadIdx.x + __cek_off) : (d) == 1 ? (long long)(blockIdx.y * blockDim.y + threadIdx.y) : (long long)(blockIdx.z * blockDim.z + threadIdx.z))
#define get_local_id(d) ((long long)((d) == 0 ? threadIdx.x : (d) == 1 ? threadIdx.y : threadIdx.z))
#define get_group_id(d) ((long long)((d) == 0 ? blockIdx.x : (d) == 1 ? blockIdx.y : blockIdx.z))
#define get_local_size(d) ((long long)((d) == 0 ? blockDim.x : (d) == 1 ? blockDim.y : blockDim.z))
#define get_global_size(d) ((d) == 0 ? __cek_gsize : (long long)((d) == 1 ? gridDim.y * blockDim.y : gridDim.z * blockDim.z))
#define get_num_groups(d) ((d) == 0 ? __cek_gsize / (long long)blockDim.x : (long long)((d) == 1 ? gridDim.y : gridDim.z))
#define get_global_offset(d) ((d) == 0 ? __cek_off : 0ll)
#define cek_global_group_id() ((long long)blockIdx.x + __cek_off / (long long)blockDim.x)
#define cek_local_group_id() ((long long)blockIdx.x)
#define cek_local_num_groups() ((long long)gridDim.x)
#ifdef CEK_OPENCL_DIALECT
typedef unsigned int uint; typedef unsigned char uchar; typedef unsigned short ushort; typedef unsigned long ulong;
__device__ inline float native_sqrt(float x) { return __fsqrt_rn(x); }
__device__ inline float native_rsqrt(float x) { return rsqrtf(x); }
__device__ inline float native_exp(float x) { return __expf(x); }
__device__ inline float native_sin(float x) { return __sinf(x); }
__device__ inline float native_cos(float x) { return __cosf(x); }
__device__ inline float native_divide(float a, float b) { return __fdividef(a, b); }
__device__ inline float mad(float a, float b, float c) { return fmaf(a, b, c); }
__device__ inline float clamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ inline int atomic_add(int* p, int v) { return atomicAdd(p, v); }
__device__ inline int atomic_inc(int* p) { return atomicAdd(p, 1); }
#endif
// ---- end prelude ----
)CEK";

static const char* kCpuPrelude = R"CEK(
// ---- cekirdekler_amd CPU prelude (host device) ----
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <tuple>
#include <ucontext.h>
#define CEK_CPU 1
struct dim3 { unsigned x = 1, y = 1, z = 1; };
static thread_local dim3 threadIdx, blockIdx, blockDim, gridDim;
static thread_local long long __cek_off = 0, __cek_gsize = 0;
// kernels are inlined into their runner's work-item loop (which the
// compiler then vectorizes across work-items); CEK_NO_FORCE_INLINE is the
// retry for a kernel that cannot be inlined
#ifndef CEK_NO_FORCE_INLINE
#define __global__ __attribute__((always_inline))
#else
#define __global__
#endif
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__
#define __restrict__ __restrict
#define __launch_bounds__(...)
#define __shared__ static thread_local
struct float2 { float x, y; }; struct float3 { float x, y, z; }; struct float4 { float x, y, z, w; };
struct int2 { int x, y; }; struct int4 { int x, y, z, w; }; struct uint2 { unsigned x, y; }; struct uint4 { unsigned x, y, z, w; };
struct double2 { double x, y; };
static inline float2 make_float2(float a, float b) { return {a, b}; }
static inline float3 make_float3(float a, float b, float c) { return {a, b, c}; }
static inline float4 make_float4(float a, float b, float c, float d) { return {a, b, c, d}; }
static inline int2 make_int2(int a, int b) { return {a, b}; }
static inline int4 make_int4(int a, int b, int c, int d) { return {a, b, c, d}; }
static inline float rsqrtf(float x) { return 1.0f / std::sqrt(x); }
static inline double rsqrt(double x) { return 1.0 / std::sqrt(x); }
static inline float __fdividef(float a, float b) { return a / b; }
static inline float __fsqrt_rn(float x) { return std::sqrt(x); }
using std::min; using std::max;
// float overloads of the math functions in the global namespace, as HIP
// provides them on the GPU: sin(float) is sinf, not sin(double) rounded
using std::sin; using std::cos; using std::tan; using std::asin; using std::acos; using std::atan;
using std::atan2; using std::sinh; using std::cosh; using std::tanh; using std::exp; using std::exp2;
using std::log; using std::log2; using std::log10; using std::pow; using std::sqrt; using std::cbrt;
using std::fabs; using std::floor; using std::ceil; using std::fmod; using std::fmin; using std::fmax;
using std::round; using std::trunc; using std::hypot;
#if defined(__GNUC__) && !defined(__clang__)
// vector variants from glibc's libmvec (since 2.22), so g++ can vectorize a
// work-item loop that calls them (clang gets the same from -fveclib=libmvec)
extern "C" float sinf(float) noexcept __attribute__((__simd__("notinbranch")));
extern "C" float cosf(float) noexcept __attribute__((__simd__("notinbranch")));
extern "C" float expf(float) noexcept __attribute__((__simd__("notinbranch")));
extern "C" float logf(float) noexcept __attribute__((__simd__("notinbranch")));
#endif
template <class T> static inline T atomicAdd(T* p, T v) {
  T old, nv; __atomic_load(p, &old, __ATOMIC_RELAXED);
  do { nv = old + v; } while (!__atomic_compare_exchange(p, &old, &nv, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST));
  return old;
}
static inline int atomicAdd(int* p, int v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
static inline unsigned atomicAdd(unsigned* p, unsigned v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
static inline long long atomicAdd(long long* p, long long v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
template <class T> static inline T atomicMax(T* p, T v) { T o = *p; while (o < v && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {} return o; }
template <class T> static inline T atomicMin(T* p, T v) { T o = *p; while (o > v && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {} return o; }
template <class T> static inline T atomicExch(T* p, T v) { return __atomic_exchange_n(p, v, __ATOMIC_SEQ_CST); }
static inline void __threadfence() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
// Work-group barrier on the CPU device: every work-item of a group is a
// fiber (ucontext) on one host thread; __syncthreads() yields to the group
// scheduler, which resumes the items round-robin.
struct __CekFibers { ucontext_t sched; ucontext_t* items; int cur; };
static thread_local __CekFibers* __cek_fib = nullptr;
static inline void __syncthreads() { if (__cek_fib) swapcontext(&__cek_fib->items[__cek_fib->cur], &__cek_fib->sched); }
// Typed call of a kernel from the runner's void* argument array: the
// parameter types come from the kernel's own signature, so the call is a
// direct call the compiler can inline into the work-item loop (and
// vectorize), not a call through a function pointer of another type.
template <unsigned long long... I> struct __CekSeq {};
template <unsigned long long N, unsigned long long... I> struct __CekMakeSeq : __CekMakeSeq<N - 1, N - 1, I...> {};
template <unsigned long long... I> struct __CekMakeSeq<0, I...> { using type = __CekSeq<I...>; };
template <class... P, unsigned long long... I>
static inline __attribute__((always_inline)) void __cek_call_i(void (*f)(P...), void** a, __CekSeq<I...>) {
  f(reinterpret_cast<P>(a[I])...);
}
template <class... P>
static inline __attribute__((always_inline)) void __cek_call(void (*f)(P...), void** a) {
  __cek_call_i(f, a, typename __CekMakeSeq<sizeof...(P)>::type{});
}
// The kernel's arguments as typed values, read from the argument array once
// per runner call: inside the work-item loop a reload of args[i] per item
// keeps the compiler from vectorizing kernels with conditional memory
// accesses (it cannot bound them against the array the pointers came from).
template <class... P, unsigned long long... I>
static inline __attribute__((always_inline)) std::tuple<P...> __cek_args_i(void (*)(P...), void** a, __CekSeq<I...>) {
  return std::tuple<P...>(reinterpret_cast<P>(a[I])...);
}
template <class... P>
static inline __attribute__((always_inline)) std::tuple<P...> __cek_args(void (*f)(P...), void** a) {
  return __cek_args_i(f, a, typename __CekMakeSeq<sizeof...(P)>::type{});
}
#define get_global_id(d) ((d) == 0 ? ((long long)blockIdx.x * (long long)blockDim.x + (long long)threadIdx.x + __cek_off) : 0ll)
#define get_local_id(d) ((long long)((d) == 0 ? threadIdx.x : 0))
#define get_group_id(d) ((long long)((d) == 0 ? blockIdx.x : 0))
#define get_local_size(d) ((long long)((d) == 0 ? blockDim.x : 1))
#define get_global_size(d) ((d) == 0 ? __cek_gsize : 1ll)
#define get_num_groups(d) ((d) == 0 ? __cek_gsize / (long long)blockDim.x : 1ll)
#define get_global_offset(d) ((d) == 0 ? __cek_off : 0ll)
#define cek_global_group_id() ((long long)blockIdx.x + __cek_off / (long long)blockDim.x)
#define cek_local_group_id() ((long long)blockIdx.x)
#define cek_local_num_groups() ((long long)gridDim.x)
#ifdef CEK_OPENCL_DIALECT
typedef unsigned int uint; typedef unsigned char uchar; typedef unsigned short ushort; typedef unsigned long ulong;
static inline float native_sqrt(float x) { return std::sqrt(x); }
static inline float native_rsqrt(float x) { return 1.0f / std::sqrt(x); }
static inline float native_exp(float x) { return std::exp(x); }
static inline float native_sin(float x) { return std::sin(x); }
static inline float native_cos(float x) { return std::cos(x); }
static inline float native_divide(float a, float b) { return a / b; }
static inline float mad(float a, float b, float c) { return a * b + c; }
static inline float clamp(float x, float lo, float hi) { return std::fmin(std::fmax(x, lo), hi); }
static inline int atomic_add(int* p, int v) { return atomicAdd(p, v); }
static inline int atomic_inc(int* p) { return atomicAdd(p, 1); }
#endif
// ---- end prelude ----
)CEK";

// ------------------------------------------------- device-side enqueue --
// OpenCL 2.0 enqueue_kernel has no HIP equivalent.  The
// MI355X-native replacement is GPU-resident: a kernel calls
//   cek_enqueue(child, n, param)
// to append a launch record {child, n, param} to its device's queue, one
// queue level deeper than itself.  Children are written as
//   __cek_child__ void child(long long id, long long param, <parent's params>)
// After the parent, the runtime issues one generated dispatcher launch per
// child level on the same stream (stream order makes each level's records
// visible to the next): the dispatcher's waves grid-stride over every record
// of its level and call the child for each id.  No host round trip, no spin
// waits; the depth is bounded (kDynLevels) and a full level or a too-deep
// enqueue counts an error the host can read.

bool uses_device_enqueue(const std::string& src) {
  static const std::regex re(R"((^|[^\w])cek_enqueue\s*\()");
  return std::regex_search(src, re);
}

static std::string param_name(const std::string& p) {
  static const std::regex re(R"(([A-Za-z_]\w*)\s*(\[[^\]]*\])?\s*$)");
  std::smatch m;
  return std::regex_search(p, m, re) ? m[1].str() : std::string();
}

static std::vector<std::string> split_params(const std::string& inside) {
  std::vector<std::string> out;
  std::string cur;
  int depth = 0;
  for (char c : inside) {
    if (c == '(' || c == '<' || c == '[') ++depth;
    if (c == ')' || c == '>' || c == ']') --depth;
    if (c == ',' && depth == 0) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  std::string t;
  for (char c : cur)
    if (!isspace(static_cast<unsigned char>(c))) t += c;
  if (!t.empty() && t != "void") out.push_back(cur);
  return out;
}

static size_t match_brace(const std::string& s, size_t open) {
  int depth = 0;
  for (size_t i = open; i < s.size(); ++i) {
    if (s[i] == '{') ++depth;
    else if (s[i] == '}') {
      if (--depth == 0) return i;
    }
  }
  return std::string::npos;
}

static std::string dyn_prelude(const std::vector<std::string>& children) {
  std::ostringstream os;
  os << "// ---- device-side enqueue ----\n"
     << "#define CEK_DYN_LEVELS " << kDynLevels << "\n#define CEK_DYN_CAP " << kDynCap << "\n"
     << "struct __CekRec { int child; int pad; long long n; long long param; };\n"
     << "struct __CekQueue { int count[8]; int errors; int pad[7]; __CekRec recs[CEK_DYN_LEVELS][CEK_DYN_CAP]; };\n"
     << "__device__ inline void __cek_enqueue(void* qv, int level, int child, long long n, long long param) {\n"
     << "  __CekQueue* q = (__CekQueue*)qv;\n"
     << "  if (n <= 0) return;\n"
     << "  if (level + 1 >= CEK_DYN_LEVELS) { atomicAdd(&q->errors, 1); return; }\n"
     << "  int slot = atomicAdd(&q->count[level + 1], 1);\n"
     << "  if (slot >= CEK_DYN_CAP) { atomicAdd(&q->errors, 1); return; }\n"
     << "  __CekRec r; r.child = child; r.pad = 0; r.n = n; r.param = param;\n"
     << "  q->recs[level + 1][slot] = r;\n"
     << "}\n"
     << "#define cek_enqueue(child, n, param) __cek_enqueue(__cek_q, __cek_level, __cek_child_##child, (long long)(n), (long long)(param))\n"
     << "#define __cek_child__ __device__\n";
  if (!children.empty()) {
    os << "enum {";
    for (size_t i = 0; i < children.size(); ++i) os << (i ? ", " : " ") << "__cek_child_" << children[i] << " = " << i;
    os << " };\n";
  }
  return os.str();
}

std::string gpu_rewrite(const std::string& src) {
  std::string s = is_opencl_dialect(src) ? translate_opencl(src) : strip_comments(src);
  // hiprtc supplies the HIP runtime itself.
  s = regex_replace_all(s, R"(#\s*include\s*[<"]hip/hip_runtime\.h[>"])", "");
  const bool dyn = uses_device_enqueue(s);
  auto sites = find_sites(s);
  // dispatchers (generated from the unmodified parameter lists)
  std::vector<std::string> children;
  std::string dispatchers;
  if (dyn) {
    static const std::regex child_re(R"(__cek_child__\s+void\s+([A-Za-z_]\w*)\s*\()");
    for (auto it = std::sregex_iterator(s.begin(), s.end(), child_re); it != std::sregex_iterator(); ++it)
      children.push_back((*it)[1].str());
    std::set<std::string> done;
    for (auto& k : sites) {
      if (!done.insert(k.sig.name).second) continue;
      size_t ob = s.find('{', k.close), cb = ob == std::string::npos ? ob : match_brace(s, ob);
      if (cb == std::string::npos || !uses_device_enqueue(s.substr(ob, cb - ob))) continue;
      const std::string inside = s.substr(k.open + 1, k.close - k.open - 1);
      const auto params = split_params(inside);
      std::string names;
      for (auto& p : params) names += ", " + param_name(p);
      std::ostringstream os;
      os << "extern \"C\" __global__ void __cek_dispatch_" << k.sig.name << "(" << inside
         << (params.empty() ? "" : ", ")
         << "long long __cek_off, long long __cek_gsize, void* __cek_q, int __cek_level) {\n"
         << "  __CekQueue* q = (__CekQueue*)__cek_q;\n"
         << "  const int cnt = min(q->count[__cek_level], CEK_DYN_CAP);\n"
         << "  const long long stride = (long long)gridDim.x * blockDim.x;\n"
         << "  for (int r = 0; r < cnt; ++r) {\n"
         << "    const __CekRec rec = q->recs[__cek_level][r];\n"
         << "    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < rec.n; i += stride) {\n"
         << "      switch (rec.child) {\n";
      for (size_t c = 0; c < children.size(); ++c)
        os << "        case " << c << ": " << children[c] << "(i, rec.param" << names
           << ", __cek_q, __cek_level); break;\n";
      os << "        default: break;\n      }\n    }\n  }\n}\n";
      dispatchers += os.str();
    }
  }
  const std::string hidden =
      dyn ? "long long __cek_off, long long __cek_gsize, void* __cek_q, int __cek_level"
          : "long long __cek_off, long long __cek_gsize";
  for (auto it = sites.rbegin(); it != sites.rend(); ++it) {
    const auto& k = *it;
    if (k.sig.arity == 0) {
      s.replace(k.open + 1, k.close - k.open - 1, hidden);
    } else {
      s.insert(k.close, ", " + hidden);
    }
    if (!k.has_extern_c) s.insert(k.global_pos, "extern \"C\" ");
  }
  if (!dyn) return std::string(kGpuPrelude) + "#line 1\n" + s;
  // children get the queue and their own level (enqueues go one deeper)
  static const std::regex child_re(R"(__cek_child__\s+void\s+([A-Za-z_]\w*)\s*\()");
  std::vector<std::pair<size_t, size_t>> parens;
  for (auto it = std::sregex_iterator(s.begin(), s.end(), child_re); it != std::sregex_iterator(); ++it) {
    size_t open = static_cast<size_t>(it->position(0) + it->length(0) - 1);
    size_t close = match_paren(s, open);
    if (close != std::string::npos) parens.emplace_back(open, close);
  }
  for (auto it = parens.rbegin(); it != parens.rend(); ++it)
    s.insert(it->second, ", void* __cek_q, int __cek_level");
  return std::string(kGpuPrelude) + dyn_prelude(children) + "#line 1\n" + s + "\n// ---- dispatchers ----\n" +
         dispatchers;
}

std::string cpu_rewrite(const std::string& src) {
  std::string s = is_opencl_dialect(src) ? translate_opencl(src) : strip_comments(src);
  s = regex_replace_all(s, R"(#\s*include\s*[<"]hip/[\w\.]+[>"])", "");
  auto sites = find_sites(s);
  for (auto it = sites.rbegin(); it != sites.rend(); ++it)
    if (!it->has_extern_c) s.insert(it->global_pos, "extern \"C\" ");
  bool barriers = std::regex_search(s, std::regex(R"(__syncthreads\s*\()"));
  std::ostringstream os;
  os << kCpuPrelude << "#line 1\n" << s << "\n// ---- runners ----\n";
  std::set<std::string> seen;
  for (auto& k : sites) {
    if (!seen.insert(k.sig.name).second) continue;
    const std::string& n = k.sig.name;
    std::string c = "__cek_call(&" + n + ", args)";
    if (!barriers) {
      // whole work-groups per outer iteration (the pool hands out multiples
      // of L), so the inner loop only advances threadIdx.x.  "omp simd"
      // (-fopenmp-simd: the pragma only, no OpenMP runtime) states what the
      // kernel model already guarantees — work-items without barriers are
      // independent — so the compiler vectorizes across work-items also
      // when the kernel body has loops of its own (it refuses "multiple
      // nested loops" otherwise and runs such kernels one item at a time)
      os << "extern \"C\" void __cek_run_" << n
         << "(void** args, long long off, long long gsize, long long first, long long count, int L) {\n"
         << "  __cek_off = off; __cek_gsize = gsize; blockDim.x = (unsigned)L;\n"
         << "  gridDim.x = (unsigned)(gsize / L);\n"
         << "  const auto __cek_a = __cek_args(&" << n << ", args);\n"
         << "  for (long long g0 = first; g0 < first + count; g0 += L) {\n"
         << "    blockIdx.x = (unsigned)((g0 - off) / L);\n"
         << "    const int n_items = (int)std::min<long long>(L, first + count - g0);\n"
         << "    _Pragma(\"omp simd\")\n"
         << "    for (int t = 0; t < n_items; ++t) { threadIdx.x = (unsigned)t; std::apply(" << n
         << ", __cek_a); }\n"
         << "  }\n}\n";
    } else {
      // Fiber runner: whole groups only (first/count multiples of L).
      os << "static thread_local void** __cek_args_" << n << ";\n"
         << "static thread_local char* __cek_done_" << n << ";\n"
         << "static void __cek_entry_" << n << "() { void** args = __cek_args_" << n << "; " << c
         << "; __cek_done_" << n << "[threadIdx.x] = 1; }\n"
         << "extern \"C\" void __cek_run_" << n
         << "(void** args, long long off, long long gsize, long long first, long long count, int L) {\n"
         << "  __cek_off = off; __cek_gsize = gsize; blockDim.x = (unsigned)L; gridDim.x = (unsigned)(gsize / L);\n"
         << "  __cek_args_" << n << " = args;\n"
         << "  const size_t stack = 64 * 1024;\n"
         << "  static thread_local char* stacks = nullptr; static thread_local int cap = 0;\n"
         << "  static thread_local ucontext_t* items = nullptr; static thread_local char* done = nullptr;\n"
         << "  if (cap < L) { delete[] stacks; delete[] items; delete[] done; stacks = new char[stack * L];\n"
         << "    items = new ucontext_t[L]; done = new char[L]; cap = L; }\n"
         << "  __cek_done_" << n << " = done;\n"
         << "  __CekFibers fib; fib.items = items; __cek_fib = &fib;\n"
         << "  for (long long g0 = first; g0 < first + count; g0 += L) {\n"
         << "    blockIdx.x = (unsigned)((g0 - off) / L);\n"
         << "    for (int t = 0; t < L; ++t) { getcontext(&items[t]); items[t].uc_stack.ss_sp = stacks + stack * t;\n"
         << "      items[t].uc_stack.ss_size = stack; items[t].uc_link = &fib.sched;\n"
         << "      makecontext(&items[t], __cek_entry_" << n << ", 0); done[t] = 0; }\n"
         << "    int remaining = L;\n"
         << "    while (remaining > 0) {\n"
         << "      for (int t = 0; t < L; ++t) { if (done[t]) continue; fib.cur = t; threadIdx.x = (unsigned)t;\n"
         << "        swapcontext(&fib.sched, &items[t]); }\n"
         << "      remaining = 0; for (int t = 0; t < L; ++t) remaining += !done[t];\n"
         << "    }\n"
         << "  }\n  __cek_fib = nullptr;\n}\n";
    }
  }
  std::string out = os.str();
  return out;
}

// ------------------------------------------------------------ compilers --

static std::mutex g_jit_mu;
static std::map<std::string, std::string> g_code_cache;

static std::string rocm_path() {
  const char* e = getenv("ROCM_PATH");
  return e && *e ? e : "/opt/rocm";
}

bool compile_gpu(const std::string& rsrc, const std::vector<std::string>& options,
                 const std::string& arch_in, std::string& code, std::string& log) {
  std::string arch = arch_in.empty() ? "gfx950" : arch_in.substr(0, arch_in.find(':'));
  std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-std=c++17",
                                   "-I" + rocm_path() + "/include"};
  for (auto& o : options) opts.push_back(o);
  std::string key_src = rsrc;
  for (auto& o : opts) key_src += "\x01" + o;
  std::string key = hash_hex(key_src);
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto it = g_code_cache.find(key);
    if (it != g_code_cache.end()) {
      code = it->second;
      return true;
    }
  }
  std::string path = cache_dir() + "/gpu_" + arch + "_" + key + ".hsaco";
  if (read_file(path, code) && !code.empty()) {
    std::lock_guard<std::mutex> g(g_jit_mu);
    g_code_cache[key] = code;
    return true;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, rsrc.c_str(), "cek_kernels.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return false;
  }
  std::vector<const char*> copts;
  for (auto& o : opts) copts.push_back(o.c_str());
  hiprtcResult r = hiprtcCompileProgram(prog, static_cast<int>(copts.size()), copts.data());
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  if (ls > 1) {
    std::string l(ls, '\0');
    hiprtcGetProgramLog(prog, &l[0]);
    l.resize(strlen(l.c_str()));
    log = l;
  }
  if (r != HIPRTC_SUCCESS) {
    if (log.empty()) log = hiprtcGetErrorString(r);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.assign(cs, '\0');
  hiprtcGetCode(prog, &code[0]);
  hiprtcDestroyProgram(&prog);
  write_file_atomic(path, code);
  std::lock_guard<std::mutex> g(g_jit_mu);
  g_code_cache[key] = code;
  return true;
}

bool compile_cpu(const std::string& rsrc, const std::vector<std::string>& options,
                 std::string& so_path, std::string& log) {
  const char* cxx_env = getenv("CEK_CXX");
  std::string cxx = cxx_env && *cxx_env ? cxx_env : "g++";
  // -ffp-contract=off: results match the host reference (numpy) bit-for-bit.
  // -fno-math-errno: sqrtf & co. need no errno branch (kernels have no
  // errno), which would otherwise keep any loop calling them scalar; the
  // results stay the correctly rounded IEEE ones.
  // -fno-semantic-interposition: the runner's call of an extern "C" kernel
  // in the same .so is a direct, inlinable call (not through the PLT), so
  // the work-item loop vectorizes; -ftls-model=local-dynamic: the work-item
  // index variables (thread_local) cost one __tls_get_addr per runner call
  // instead of one per work item.
  std::string flags =
      "-O3 -march=native -ffp-contract=off -fPIC -shared -std=c++17 -w -fno-semantic-interposition "
      "-ftls-model=local-dynamic -fopenmp-simd -fno-math-errno";
  for (auto& o : options) flags += " " + o;
  // "vplan": the build may fall back to clang (below); part of the key so a
  // cache entry from before that fallback existed is not reused
  std::string key = hash_hex(rsrc + "\x01" + cxx + "\x01" + flags + "\x01vplan-libmvec");
  std::string dir = cache_dir();
  so_path = dir + "/cpu_" + key + ".so";
  struct stat st;
  if (stat(so_path.c_str(), &st) == 0 && st.st_size > 0) return true;
  std::lock_guard<std::mutex> g(g_jit_mu);
  std::string src_path = dir + "/cpu_" + key + "." + std::to_string(getpid()) + ".cpp";
  std::string tmp_so = so_path + ".tmp." + std::to_string(getpid());
  std::string log_path = src_path + ".log";
  write_file_atomic(src_path, rsrc);
  // With the default g++ the vectorizer's report says whether any loop was
  // vectorized.  g++ vectorizes the work-item loop around a kernel with a
  // loop of its own only when the body has no other control flow ("if (i >=
  // n) return;" keeps it scalar); when it vectorized nothing, the kernel is
  // rebuilt with clang's outer-loop vectorizer (VPlan native path), which
  // handles those bodies (per 4 M items, one thread: a 24-step FMA loop plus
  // a branch 99 -> 8.8 ms, a guard "if (i >= n) return;" before a 16-step
  // loop 32 -> 4.1 ms; bit-identical results).  g++ stays first: on kernels
  // it does vectorize it is faster (all-pairs n-body 2.2 vs 3.5 ms).
  const bool auto_cxx = !(cxx_env && *cxx_env);
  const std::string vec_path = src_path + ".vec";
  std::string cmd = cxx + " " + flags + (auto_cxx ? " -fopt-info-vec-optimized=" + vec_path : std::string()) +
                    " -o " + tmp_so + " " + src_path + " > " + log_path + " 2>&1";
  int rc = std::system(cmd.c_str());
  if (rc != 0) {  // a kernel the compiler cannot inline: build it as a call
    const std::string retry = cxx + " " + flags + " -DCEK_NO_FORCE_INLINE -o " + tmp_so + " " + src_path + " > " +
                              log_path + " 2>&1";
    rc = std::system(retry.c_str());
  } else if (auto_cxx && rsrc.find("__cek_fib = &fib") == std::string::npos) {
    std::string report;
    read_file(vec_path, report);
    const char* rocm = getenv("ROCM_PATH");
    const std::string clang = std::string(rocm && *rocm ? rocm : "/opt/rocm") + "/llvm/bin/clang++";
    if (report.find("vectorized") == std::string::npos && stat(clang.c_str(), &st) == 0) {
      // -fveclib=libmvec: math calls in the loop use glibc's vector
      // variants; the build is kept only if it loads (every libmvec symbol
      // it names exists here), else rebuilt without it
      const std::string tmp2 = tmp_so + ".vplan";
      for (const char* veclib : {" -fveclib=libmvec", ""}) {
        const std::string alt = clang + " " + flags + veclib + " -mllvm -enable-vplan-native-path -o " + tmp2 + " " +
                                src_path + " > /dev/null 2>&1";
        if (std::system(alt.c_str()) != 0) continue;
        void* h = dlopen(tmp2.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        dlclose(h);
        rename(tmp2.c_str(), tmp_so.c_str());
        break;
      }
      unlink(tmp2.c_str());
    }
  }
  unlink(vec_path.c_str());
  read_file(log_path, log);
  unlink(log_path.c_str());
  unlink(src_path.c_str());
  if (rc != 0) {
    unlink(tmp_so.c_str());
    if (log.empty()) log = "host compiler failed: " + cmd;
    return false;
  }
  rename(tmp_so.c_str(), so_path.c_str());
  return true;
}

// ---------------------------------------------------------------- Program --

std::shared_ptr<Program> Program::build(const DeviceInfo& dev, const std::string& src,
                                        const std::vector<std::string>& options,
                                        const std::vector<std::string>& prebuilt) {
  auto p = std::shared_ptr<Program>(new Program());
  p->type_ = dev.type;
  double t0 = now_ms();
  p->kernels_ = src.empty() ? std::vector<KernelSig>{} : parse_kernels(src);
  if (dev.type == kGPU) {
    CEK_HIP(hipSetDevice(dev.ordinal));
    if (!src.empty()) {
      std::string code, log;
      if (!compile_gpu(gpu_rewrite(src), options, dev.arch, code, log)) {
        p->log_ = log;
        return p;
      }
      p->log_ = log;
      hipModule_t m;
      CEK_HIP(hipModuleLoadData(&m, code.data()));
      p->modules_.push_back(m);
      for (auto& k : p->kernels_) {
        hipFunction_t f;
        CEK_HIP(hipModuleGetFunction(&f, m, k.name.c_str()));
        p->gpu_fns_[k.name] = f;
      }
      p->dynamic_ = uses_device_enqueue(src);
      if (p->dynamic_)
        for (auto& k : p->kernels_) {
          hipFunction_t f;
          const std::string dn = "__cek_dispatch_" + k.name;
          if (hipModuleGetFunction(&f, m, dn.c_str()) == hipSuccess) {
            p->gpu_fns_[dn] = f;
            p->dispatchers_.insert(k.name);
          } else {
            (void)hipGetLastError();
          }
        }
    }
    // prebuilt entries: "path|name1,name2"
    for (auto& pb : prebuilt) {
      auto bar = pb.find('|');
      std::string path = pb.substr(0, bar);
      std::string names = bar == std::string::npos ? "" : pb.substr(bar + 1);
      hipModule_t m;
      CEK_HIP(hipModuleLoad(&m, path.c_str()));
      p->modules_.push_back(m);
      std::stringstream ss(names);
      std::string n;
      while (std::getline(ss, n, ',')) {
        if (n.empty()) continue;
        int arity = -1;  // "name:arity" declares the array-parameter count
        auto colon = n.find(':');
        if (colon != std::string::npos) {
          arity = std::stoi(n.substr(colon + 1));
          n = n.substr(0, colon);
        }
        hipFunction_t f;
        CEK_HIP(hipModuleGetFunction(&f, m, n.c_str()));
        p->gpu_fns_[n] = f;
        p->kernels_.push_back({n, arity});
      }
    }
  } else {
    if (uses_device_enqueue(src)) {
      p->log_ = "cek_enqueue (device-side enqueue) runs on GPU devices only";
      return p;
    }
    if (!src.empty()) {
      std::string so, log;
      if (!compile_cpu(cpu_rewrite(src), options, so, log)) {
        p->log_ = log;
        return p;
      }
      p->log_ = log;
      p->dl_ = dlopen(so.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (!p->dl_) {
        p->log_ = std::string("dlopen failed: ") + dlerror();
        return p;
      }
      for (auto& k : p->kernels_) {
        void* f = dlsym(p->dl_, ("__cek_run_" + k.name).c_str());
        if (!f) {
          p->log_ += "missing runner for " + k.name + "\n";
          return p;
        }
        p->cpu_fns_[k.name] = reinterpret_cast<CpuRunner>(f);
      }
    }
  }
  if (p->kernels_.empty()) {
    p->log_ += "no kernel found in source (expected `__global__ void name(...)`)";
    return p;
  }
  p->build_ms_ = now_ms() - t0;
  p->ok_ = true;
  return p;
}

Program::~Program() {
  for (auto m : modules_) (void)hipModuleUnload(m);
  // dlclose intentionally skipped: thread_local destructors in the kernel
  // object may still be registered on pool threads.
}

int Program::arity(const std::string& name) const {
  std::lock_guard<std::mutex> g(arity_mu_);
  if (arity_.size() != kernels_.size()) {
    arity_.clear();
    for (const auto& k : kernels_) arity_.emplace(k.name, k.arity);
  }
  auto it = arity_.find(name);
  return it == arity_.end() ? -1 : it->second;
}

bool Program::has(const std::string& name) const {
  return type_ == kGPU ? gpu_fns_.count(name) > 0 : cpu_fns_.count(name) > 0;
}

hipFunction_t Program::gpu_fn(const std::string& name) const {
  auto it = gpu_fns_.find(name);
  if (it == gpu_fns_.end()) throw Error("kernel not found: " + name);
  return it->second;
}

CpuRunner Program::cpu_fn(const std::string& name) const {
  auto it = cpu_fns_.find(name);
  if (it == cpu_fns_.end()) throw Error("kernel not found on CPU device: " + name);
  return it->second;
}

}  // namespace cek

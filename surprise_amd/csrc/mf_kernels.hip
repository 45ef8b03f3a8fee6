// mf_kernels.hip -- CDNA4 (gfx950) kernels for Surprise's SVD / SVD++ SGD training path.
//
// Replaces the per-rating Cython loops of nickmvincent/Surprise
//   SVD.sgd    surprise/prediction_algorithms/matrix_factorization.pyx:241-262
//   SVDpp.sgd  surprise/prediction_algorithms/matrix_factorization.pyx:463-498
// and the batched form of SVD.estimate / SVDpp.estimate (:269-299, :506-522).
//
// Execution model (see DESIGN.md for the full argument):
//   * one 64-lane wavefront owns one user at a time (users taken from `sched`, heaviest first,
//     strided over all wavefronts of the grid).  pu[u] and bu[u] live in registers for the whole
//     user block, so the user side is race-free and follows the reference's per-rating order;
//   * the item rows qi[i] / bi[i] (and yj for SVD++) are the shared, lock-free Hogwild! state;
//   * a factor row is spread over the wave "strided": lane l holds elements l, l+64, l+128, ...
//     so every gather/scatter instruction touches 64 consecutive dwords (256 B) of one row;
//   * the user's (item, rating) stream is read with scalar loads two groups ahead, and the item
//     rows of the next kPF ratings are gathered ahead of use (software pipeline), so the
//     dependent chain per rating is register-only: FMA partials -> DPP/permlane wave reduction
//     -> error -> FMA updates;
//   * the dot product is reduced with 4 DPP row ops + v_permlane16_swap + v_permlane32_swap
//     (no LDS round trip), leaving the sum in every lane.
// No MFMA: the path is gather/scatter-bound.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <mutex>
#include <type_traits>

#include "../../include/surprise_amd.h"

// Build layout: this file is compiled once as the main translation unit (everything but the
// epoch kernels) and once per (dtype, mode, SVD/SVD++) with -DMF_TU_EPOCH -DMF_INST_T=...
// -DMF_INST_M=... -DMF_INST_PP=..., each of those defining only mf_ext::launch_epoch_tm for
// its combination (surprise_amd/build.py compiles the units in parallel and links them).
namespace mf_ext {
extern thread_local char g_err[256];
template <typename T, int M, bool PP>
int launch_epoch_tm(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                    int32_t ldu, void *qb, int32_t ldq, void *yj, void *qlog, void *elog, int32_t K,
                    int32_t biased, const mf_hyper_t *hp, int64_t waves, bool dups, int xmask,
                    int hx, double *psq, int err_col, int ck_ld, int32_t *status,
                    const uint8_t *hot, const int64_t *urow, bool nt, const int32_t *crow,
                    void *stream);
// this unit's g_dispatch_sum (the dispatch check of the masked launches it holds)
template <typename T, int M, bool PP>
int dispatch_sum_tm(unsigned long long *out);
}  // namespace mf_ext

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves per workgroup
#ifndef MF_PF
#define MF_PF 8
#endif
constexpr int kPF = MF_PF;   // item rows gathered ahead of use


using mf_ext::g_err;

int set_err(int code, const char *msg) {
    snprintf(g_err, sizeof(g_err), "%s (code %d)", msg, code);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

int grid_for_waves(int64_t waves) {
    int64_t blocks = (waves * kWave + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

// blocks giving `waves` wave slots on the XCDs of xmask (wave_slot): a multiple of 8
int grid_for_waves_x(int64_t waves, int xmask) {
    if (!(xmask & 0xFF)) return grid_for_waves(waves);
    const int64_t per = (grid_for_waves(waves) + __builtin_popcount(xmask & 0xFF) - 1) /
                        __builtin_popcount(xmask & 0xFF);
    return (int)(8 * per);
}

// G = 8-byte lane groups per row = ceil(ld * sizeof(T) / 512) (the epoch kernel's layout)
template <typename T, typename F>
int dispatch_g(int ld, F &&f)
{
    const int g = (int)(((int64_t)ld * sizeof(T) + 511) / 512);
    if (g <= 1) return f(std::integral_constant<int, 1>{});
    if (g <= 2) return f(std::integral_constant<int, 2>{});
    if (g <= 3) return f(std::integral_constant<int, 3>{});
    if (g <= 4) return f(std::integral_constant<int, 4>{});
    if (g <= 5) return f(std::integral_constant<int, 5>{});
    return set_err(MF_E_ARG, "n_factors/ld too large");
}

template <typename T>
struct Hyper {
    T lr_bu, lr_bi, lr_pu, lr_qi, lr_yj, reg_bu, reg_bi, reg_pu, reg_qi, reg_yj, gm;
};

// x^n by repeated squaring (n >= 0)
template <typename T>
__device__ __forceinline__ T pow_int(T x, int n) {
    T r = T(1);
    while (n) {
        if (n & 1) r *= x;
        x *= x;
        n >>= 1;
    }
    return r;
}

template <typename T>
Hyper<T> cast_hyper(const mf_hyper_t *h) {
    Hyper<T> o;
    o.lr_bu = (T)h->lr_bu; o.lr_bi = (T)h->lr_bi; o.lr_pu = (T)h->lr_pu; o.lr_qi = (T)h->lr_qi;
    o.lr_yj = (T)h->lr_yj; o.reg_bu = (T)h->reg_bu; o.reg_bi = (T)h->reg_bi;
    o.reg_pu = (T)h->reg_pu; o.reg_qi = (T)h->reg_qi; o.reg_yj = (T)h->reg_yj;
    o.gm = (T)h->global_mean;
    return o;
}

// ---------------------------------------------------------------- wavefront primitives

// (bound_ctrl: a lane whose source lane is out of its row reads 0 -- the permutations below stay
// inside a row, row_bcast:15 has no source for row 0 -- so the compiler needs no old value: no
// v_mov of a zero before every 32-bit DPP move, which for fp64 sums was 2 of every 5 instructions)
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

// 32-bit lane exchange pattern applied to a float / double.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, dpp_i32<CTRL>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    long long b = __builtin_bit_cast(long long, v);
    int lo = dpp_i32<CTRL>((int)(b & 0xffffffffll));
    int hi = dpp_i32<CTRL>((int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// Sum of the 16-lane rows pairwise (rows 0+1, 2+3) and of the two 32-lane halves, gfx950 swaps.
__device__ __forceinline__ float swap16_add(float v) {
    auto s = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                              false, false);
    return __builtin_bit_cast(float, (int)s[0]) + __builtin_bit_cast(float, (int)s[1]);
}
__device__ __forceinline__ float swap32_add(float v) {
    auto s = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                              false, false);
    return __builtin_bit_cast(float, (int)s[0]) + __builtin_bit_cast(float, (int)s[1]);
}
__device__ __forceinline__ double swap16_add(double v) {
    long long b = __builtin_bit_cast(long long, v);
    int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    double a = __builtin_bit_cast(double, ((long long)(int)sh[0] << 32) | (unsigned int)sl[0]);
    double c = __builtin_bit_cast(double, ((long long)(int)sh[1] << 32) | (unsigned int)sl[1]);
    return a + c;
}
__device__ __forceinline__ double swap32_add(double v) {
    long long b = __builtin_bit_cast(long long, v);
    int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    auto sl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto sh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    double a = __builtin_bit_cast(double, ((long long)(int)sh[0] << 32) | (unsigned int)sl[0]);
    double c = __builtin_bit_cast(double, ((long long)(int)sh[1] << 32) | (unsigned int)sl[1]);
    return a + c;
}

// Full 64-lane sum, result broadcast to every lane. Must be called with all 64 lanes active.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    v = swap16_add(v);
    v = swap32_add(v);
    return v;
}

__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double readlane(double v, int l) {
    long long b = __builtin_bit_cast(long long, v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ int xcc_id() {
    // HW_REG_XCC_ID (hwreg 20), bits [3:0]: the XCD this wave runs on (mf_selftest_xcc: blocks
    // are dealt to the 8 XCDs round-robin).
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 0xF);
}

// ---- the dispatch check of XCD-masked launches (mf_dispatch_check)
// A masked launch numbers its waves from blockIdx and XCC_ID (wave_slot below), assuming every
// group of 8 consecutive workgroups lands on 8 distinct XCDs (verified once per device on an
// idle GPU by xcd_layout_ok).  Every masked launch also proves it as it runs: a wave (workgroup,
// mf_svd_gram_kernel) owes mix(g) for its own grid index g when g < n_slots -- blockIdx only,
// whatever XCD it runs on -- and pays back mix(slot) for the slot it took, in ONE no-return
// 64-bit vector atomic when it exits (SlotSettle), into one of kDispatchShards counters of this
// code object (each on a 128-B line of its own: no single hot word).  The slots of a launch are a
// permutation of [0, n_slots) exactly when the assumption held; then the launch leaves the
// shards' total unchanged, while a slot taken twice or never (users trained twice / never)
// leaves it nonzero.  The engine reads the total when it copies factors back and reports it.
constexpr int kDispatchShards = 256;
__device__ unsigned long long g_dispatch_sum[kDispatchShards * 16];  // (stays 0 in total)

__device__ __forceinline__ unsigned long long dispatch_mix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;  // splitmix64's finalizer
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// one lane per wave (or workgroup): its debt for grid index g, its payment for slot (-1: none)
__device__ __forceinline__ void dispatch_settle(int64_t g, int64_t slot, int64_t n_slots) {
    unsigned long long d = g < n_slots ? 0ull - dispatch_mix((uint64_t)g) : 0ull;
    if (slot >= 0) d += dispatch_mix((uint64_t)slot);
    if (d) atomicAdd(&g_dispatch_sum[(g % kDispatchShards) * 16], d);
}

// A participating wave's settlement, made when it leaves its scope (every return path of the
// kernel body): at the end, so the atomic never sits in front of the body's counted vmcnt waits.
// (host) this code object's total over the shards; 0 on success
int dispatch_sum_here(unsigned long long *out)
{
    static unsigned long long h[kDispatchShards * 16];
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dispatch_sum), sizeof(h)) != hipSuccess) return -1;
    unsigned long long t = 0;
    for (int i = 0; i < kDispatchShards; ++i) t += h[i * 16];
    *out = t;
    return 0;
}

struct SlotSettle {
    int64_t g, slot, n;
    bool on;
    __device__ SlotSettle(int xmask, int64_t slot_, int64_t n_, int64_t g_)
        : g(g_), slot(slot_), n(n_), on(xmask != 0) {}
    __device__ ~SlotSettle() {
        if (on) dispatch_settle(g, slot, n);
    }
};

// The calling wave's slot among the launch's waves on the XCDs of xmask (bit x: XCD x; 0: every
// XCD), and the number of such slots.  Blocks are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, checked by mf_selftest_xcc), so every group of 8 consecutive blocks holds
// one block per XCD: slot = ((b / 8) * c + rank of the wave's XCD in xmask) * 4 + wave in block,
// c = popcount(xmask).  Launches with a mask have a multiple of 8 blocks (grid_for_waves_x).
// Returns false for a wave on an XCD outside the mask (it settles its debt and exits); a wave
// that returns true settles through a SlotSettle(xmask, slot, n_slots, wave_grid_index()).
__device__ __forceinline__ int64_t wave_grid_index() {
    return (int64_t)blockIdx.x * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
}
__device__ __forceinline__ bool wave_slot(int xmask, int64_t &slot, int64_t &n_slots) {
    const int64_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if (!xmask) {
        slot = (int64_t)blockIdx.x * (kBlock / kWave) + w;
        n_slots = ((int64_t)gridDim.x * kBlock) / kWave;
        return true;
    }
    const int x = __builtin_amdgcn_readfirstlane(xcc_id());
    const int c = __builtin_popcount(xmask), rank = __builtin_popcount(xmask & ((1 << x) - 1));
    n_slots = (int64_t)(gridDim.x >> 3) * c * (kBlock / kWave);
    if (!((xmask >> x) & 1)) {
        slot = -1;
        if ((threadIdx.x & (kWave - 1)) == 0) dispatch_settle(wave_grid_index(), -1, n_slots);
        return false;
    }
    slot = ((int64_t)(blockIdx.x >> 3) * c + rank) * (kBlock / kWave) + w;
#ifdef MF_DISPATCH_FAULT_TEST
    if (slot == 1) slot = 0;  // (test build: slot 0 taken twice, slot 1 never -- must be reported)
#endif
    return true;
}

// ---------------------------------------------------------------- buffer (SRSRC) memory ops
//
// Every load/store/atomic of the SGD pipeline goes through a buffer descriptor.  A lane that
// must not touch memory (a factor column beyond the row, an item row of a masked "tail"
// rating) gets a byte offset >= the table's size: the hardware range check turns its load into 0 and drops
// its store, so the instruction stream has no exec-masked branches and every loop iteration
// issues the same number of memory instructions -- which lets the compiler keep the row
// prefetches of the next kPF ratings in flight behind counted vmcnt waits.

using rsrc_t = __amdgpu_buffer_rsrc_t;
// Range check, measured on gfx950 (tools/probe_buffer_range.hip): a lane's access is dropped iff
// voffset + soffset >= num_records, the sum taken without 32-bit wrap-around, for any
// num_records up to 0xFFFFFFFF.  A masked offset is a real offset plus the table size, computed
// in 32 bits here, so tables must stay below 2^31 bytes (kMaxTable, less one 4 KiB row).
constexpr uint64_t kMaxTable = 0x80000000ull - 4096;
constexpr int kSc1 = 16;                // gfx950 cache policy: sc1 (bypass the CU's L1)
constexpr int kNt = 2;                  // gfx950 cache policy: nt (streamed: not kept in L2 / MALL)

__device__ __forceinline__ rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void *q = (void *)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                             0x00020000);
}

template <typename T>
struct Buf;

template <>
struct Buf<float> {
    template <int AUX>
    __device__ static __forceinline__ float ld(rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void st(rsrc_t r, uint32_t off, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX);
    }
    __device__ static __forceinline__ void add(rsrc_t r, float *, uint32_t, uint32_t off, float v) {
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, off, 0, 0);  // memory-side add
    }
    template <int AUX>
    __device__ static __forceinline__ float lds(rsrc_t r, uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void sts(rsrc_t r, uint32_t voff, uint32_t soff, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, AUX);
    }
};

template <>
struct Buf<double> {
    template <int AUX>
    __device__ static __forceinline__ double ld(rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void st(rsrc_t r, uint32_t off, double v) {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r,
            off, 0, AUX);
    }
    // no buffer form of the f64 add: a predicated global atomic on the same bytes
    __device__ static __forceinline__ void add(rsrc_t, double *base, uint32_t bytes, uint32_t off,
                                               double v) {
        if (off < bytes) atomicAdd(base + off / sizeof(double), v);
    }
    template <int AUX>
    __device__ static __forceinline__ double lds(rsrc_t r, uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void sts(rsrc_t r, uint32_t voff, uint32_t soff, double v) {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r,
            voff, soff, AUX);
    }
};

// ---------------------------------------------------------------- SGD epoch kernel (SVD, SVD++)

enum { kPlain = MF_MODE_PLAIN, kAtomic = MF_MODE_ATOMIC, kLog = MF_MODE_LOG };

// Log rows: a lane whose column is past the bias column stores to this offset (beyond any user's
// log segment, which is < 2^30 bytes) and is dropped by the range check.
constexpr uint32_t kLogOob = 0x40000000u;

// ---- 8-byte lane elements.  A lane owns 8 consecutive bytes of a row per group v: two fp32
// columns (a float2: packed v_pk_fma_f32 / v_pk_mul_f32 math, one dwordx2 load per row) or one
// fp64 column.  Lane l, group v holds columns (l + 64 v) * W .. + W-1; a row of ld elements
// spans G = ceil(ld * sizeof(T) / 512) groups.
template <typename T>
struct Lane8;

template <>
struct Lane8<float> {
    typedef float vec __attribute__((ext_vector_type(2)));
    static constexpr int W = 2;
    __device__ static __forceinline__ vec splat(float x) { return vec{x, x}; }
    __device__ static __forceinline__ float hsum(vec v) { return v.x + v.y; }
    __device__ static __forceinline__ float get(vec v, int e) { return e ? v.y : v.x; }
    __device__ static __forceinline__ void set(vec &v, int e, float x) {
        if (e) v.y = x; else v.x = x;
    }
    template <int AUX>
    __device__ static __forceinline__ vec ld(rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void st(rsrc_t r, uint32_t off, vec v) {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r,
            off, 0, AUX);
    }
    __device__ static __forceinline__ void add(rsrc_t r, void *, uint32_t, uint32_t off, vec v) {
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v.x, r, off, 0, 0);  // memory-side adds
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v.y, r, off + 4, 0, 0);
    }
    // voffset + soffset forms (soffset: a wave-uniform row offset in an SGPR)
    template <int AUX>
    __device__ static __forceinline__ vec lds(rsrc_t r, uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void sts(rsrc_t r, uint32_t voff, uint32_t soff, vec v) {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r,
            voff, soff, AUX);
    }
    __device__ static __forceinline__ void adds(rsrc_t r, void *, uint32_t, uint32_t voff,
                                                uint32_t soff, vec v) {
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v.x, r, voff, soff, 0);
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v.y, r, voff + 4, soff, 0);
    }
};

template <>
struct Lane8<double> {
    typedef double vec;
    static constexpr int W = 1;
    __device__ static __forceinline__ vec splat(double x) { return x; }
    __device__ static __forceinline__ double hsum(vec v) { return v; }
    __device__ static __forceinline__ double get(vec v, int) { return v; }
    __device__ static __forceinline__ void set(vec &v, int, double x) { v = x; }
    template <int AUX>
    __device__ static __forceinline__ vec ld(rsrc_t r, uint32_t off) { return Buf<double>::ld<AUX>(r, off); }
    template <int AUX>
    __device__ static __forceinline__ void st(rsrc_t r, uint32_t off, vec v) { Buf<double>::st<AUX>(r, off, v); }
    __device__ static __forceinline__ void add(rsrc_t r, void *base, uint32_t bytes, uint32_t off,
                                               vec v) {
        Buf<double>::add(r, (double *)base, bytes, off, v);
    }
    template <int AUX>
    __device__ static __forceinline__ vec lds(rsrc_t r, uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
    }
    template <int AUX>
    __device__ static __forceinline__ void sts(rsrc_t r, uint32_t voff, uint32_t soff, vec v) {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r,
            voff, soff, AUX);
    }
    __device__ static __forceinline__ void adds(rsrc_t r, void *base, uint32_t bytes, uint32_t voff,
                                                uint32_t soff, vec v) {
        Buf<double>::add(r, (double *)base, bytes, voff + soff, v);
    }
};

// Full 64-lane sum returned as a wave-uniform value (scalar register): 4 DPP butterfly steps
// leave every lane with its 16-lane row sum, two DPP row broadcasts fold rows 0..3 into lane 63,
// one v_readlane.  (gfx9 DPP: row_bcast:15 = 0x142, row_bcast:31 = 0x143.)
__device__ __forceinline__ float wave_sum_u(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142,
                                                               0xA, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143,
                                                               0xC, 0xF, false));
    return readlane(v, 63);
}
__device__ __forceinline__ double wave_sum_u(double v) { return readlane(wave_sum(v), 0); }

// ---- one-element-per-lane ("Lane1") view of a row, for the float atomics: an atomic
// instruction then covers 64 consecutive dwords (256 B) instead of every other dword of 512 B.
// Lane1 group u, lane l holds column l + 64 u; for fp32 it has 2G groups, for fp64 it is the
// Lane8 layout itself.  Conversions are ds_bpermute lane exchanges (no LDS storage).
template <typename T, int G>
struct Lane1 {
    static constexpr int U = Lane8<T>::W * G;
    typedef T type[U];
};

__device__ __forceinline__ float bperm(int src_lane, float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane << 2, __builtin_bit_cast(int, x)));
}

template <int G>
__device__ __forceinline__ void to_lane1(const typename Lane8<float>::vec (&x)[G], float (&y)[2 * G]) {
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int u = 0; u < 2 * G; ++u) {  // column c = lane + 64 u lives in Lane8 group u/2, lane c/2
        const int src = 32 * (u & 1) + (lane >> 1);
        const float a = bperm(src, x[u >> 1].x), b = bperm(src, x[u >> 1].y);
        y[u] = (lane & 1) ? b : a;
    }
}
template <int G>
__device__ __forceinline__ void to_lane1(const double (&x)[G], double (&y)[G]) {
#pragma unroll
    for (int u = 0; u < G; ++u) y[u] = x[u];
}

template <int G>
__device__ __forceinline__ void to_lane8(const float (&y)[2 * G], typename Lane8<float>::vec (&x)[G]) {
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int v = 0; v < G; ++v) {  // column 2 (lane + 64 v) + e lives in Lane1 group 2v + (lane >= 32)
        const int s0 = (2 * lane) & (kWave - 1);
        const float lo0 = bperm(s0, y[2 * v]), hi0 = bperm(s0, y[2 * v + 1]);
        const float lo1 = bperm(s0 + 1, y[2 * v]), hi1 = bperm(s0 + 1, y[2 * v + 1]);
        x[v].x = lane < 32 ? lo0 : hi0;
        x[v].y = lane < 32 ? lo1 : hi1;
    }
}
// memory-side float add of one element per lane at voff + soff (rows out of range dropped)
__device__ __forceinline__ void atom_add1(rsrc_t r, void *, uint32_t, uint32_t voff, uint32_t soff,
                                          float v) {
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, voff, soff, 0);
}
__device__ __forceinline__ void atom_add1(rsrc_t, void *base, uint32_t bytes, uint32_t voff,
                                          uint32_t soff, double v) {
    if (voff + soff < bytes) atomicAdd((double *)base + (voff + soff) / sizeof(double), v);
}

template <int G>
__device__ __forceinline__ void to_lane8(const double (&y)[G], double (&x)[G]) {
#pragma unroll
    for (int v = 0; v < G; ++v) x[v] = y[v];
}

// Item table row (ldq elements): [q_0 .. q_{K-1} | b_i | 0 ...].  The user row is extended in
// registers with a constant 1 in column K, so <q_aug, p_aug> = <q_i, p_u> + b_i and the item
// bias rides in the same gather / scatter as the item factors; its update
// b_i += lr_bi (err * 1 - reg_bi b_i) is the factor rule with the per-column (lr, reg) swapped.
//
// MODE decides what happens to the item row after a rating:
//   kPlain  store q_i + d (lock-free Hogwild!; with one wave: the exact sequential reference);
//   kAtomic memory-side float add of d;
//   kLog    the item table is a read-only snapshot for the whole epoch-chunk and the rating's
//           gradient g = err pe (d = lr o (g - reg o q)) goes to row k of the delta log (k = the
//           rating's CSR position); mf_log_reduce / mf_log_apply fold the log into the table
//           afterwards (q += w o lr o (sum g - N reg o q)).  Race-free, independent of scheduling.
// SVD++'s y_j rows are shared state in every mode (kPlain: stores, kAtomic / kLog: float adds).
//
// Per rating the dependent chain is: p -> <q, p> partial (packed mul) -> wave sum -> err ->
// (lr err) -> p' = (lr err) q + (1 - lr reg) p (one packed FMA); everything that does not need
// err ((1 - lr reg) p, -lr reg q, the next row's address) is computed off that chain.
template <typename T, int G, int MODE, bool PP, bool DUPS, int kPF>
__device__ __forceinline__ void epoch_body(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, int ldu, T *qb, int ldq, T *yj, T *qlog, T *ycbuf,
    int K, int biased, Hyper<T> hp, int n_items, int64_t n_waves_req, int xmask)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    const int lane = threadIdx.x & (kWave - 1);
    // wave id through readfirstlane: the compiler then knows it (and every user index, CSR
    // bound and loop counter derived from it) is wave-uniform -> SGPRs, scalar loads, scalar
    // branches instead of exec-masked ones.
    int64_t wave, grid_waves;
    if (!wave_slot(xmask, wave, grid_waves)) return;
    SlotSettle settle((threadIdx.x & (kWave - 1)) == 0 ? xmask : 0, wave, grid_waves,
                      wave_grid_index());
    const int64_t n_waves = n_waves_req < grid_waves ? n_waves_req : grid_waves;
    if (wave >= n_waves) return;  // whole wave exits (a 1-wave launch still uses a 4-wave block)

    const uint32_t qrow = (uint32_t)ldq * sizeof(T), yrow = (uint32_t)ldu * sizeof(T);
    const uint32_t q_oob = (uint32_t)n_items * qrow, y_oob = (uint32_t)n_items * yrow;
    constexpr bool ATOM = MODE == kAtomic;  // item updates as float atomics
    constexpr bool LOG = MODE == kLog;      // item updates to the delta log
    constexpr bool YATOM = MODE != kPlain;  // SVD++ y_j updates as float atomics
    // Rows other waves are updating are read around the CU's L1 (sc1).  kPlain (the
    // deterministic one-wave path) and the kLog snapshot use plain, L1-cached loads.
    constexpr int kLdAux = MODE == kAtomic ? kSc1 : 0;
    constexpr int kYLdAux = MODE == kPlain ? 0 : kSc1;

    // per-lane constants of group v (byte offsets of the lane's 8 bytes; masked lanes get an
    // offset past the table / log so their loads read 0 and their stores are dropped)
    uint32_t cq[G], cu[G], cl[G];
    vec one[G], lrq[G], nrq[G], lrp[G], ap[G], lry[G];
    constexpr int U = Lane1<T, G>::U;  // Lane1 groups (atomics, SVD++ y rows)
    uint32_t cq1[U], cy1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = lane + kWave * u;
        cq1[u] = c < ldq ? (uint32_t)c * sizeof(T) : (uint32_t)n_items * ldq * sizeof(T);
        cy1[u] = c < ldu ? (uint32_t)c * sizeof(T) : (uint32_t)n_items * ldu * sizeof(T);
    }
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;  // first column of this lane's 8 bytes
        const uint32_t b = (uint32_t)c0 * sizeof(T);
        cq[v] = c0 < ldq ? b : q_oob;
        cu[v] = c0 < ldu ? b : (PP ? y_oob : yrow);  // >= pu record too
        // log rows are stored whole, zero padding included: a user's log segment is then one
        // contiguous, fully written byte range (partially written lines cost a read-modify-write
        // at the memory side: measured 2 TB/s effective with the padding left unwritten)
        cl[v] = c0 < ldq ? b : kLogOob;
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const int c = c0 + e;
            const bool fac = c < K, bias = biased && c == K;
            const T lq = fac ? hp.lr_qi : (bias ? hp.lr_bi : T(0));
            const T rq = fac ? hp.reg_qi : (bias ? hp.reg_bi : T(0));
            const T lp = fac ? hp.lr_pu : T(0);
            const T rp = fac ? hp.reg_pu : T(0);
            L::set(one[v], e, bias ? T(1) : T(0));
            L::set(lrq[v], e, lq);
            L::set(nrq[v], e, -lq * rq);      // d = (lr err) pe - lr reg q
            L::set(lrp[v], e, lp);
            L::set(ap[v], e, T(1) - lp * rp);  // p' = (lr err) q + (1 - lr reg) p
            L::set(lry[v], e, fac ? hp.lr_yj : T(0));
        }
    }
    const T lr_bu = biased ? hp.lr_bu : T(0);
    const T abu = T(1) - lr_bu * hp.reg_bu;
    const T decay = T(1) - hp.lr_yj * hp.reg_yj;

    const rsrc_t q_rs = make_rsrc(qb, q_oob);
    const rsrc_t y_rs = PP ? make_rsrc(yj, y_oob) : q_rs;
    // sched lists users heaviest first: its head's degree scales the priority levels
    const int prio_len = (int)(row_ptr[sched[0] + 1] - row_ptr[sched[0]]);

    // one user block: the reference's per-rating order for user u
    auto do_user = [&](const int u) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);  // |I_u| (< 2^31)
        if (n <= 0) return;
        // The epoch ends when the longest user chain ends: the waves of the heaviest users
        // take issue priority over the light users sharing their SIMD.
        if (n * 2 > prio_len) __builtin_amdgcn_s_setprio(3);
        else if (n * 4 > prio_len) __builtin_amdgcn_s_setprio(2);
        else if (n * 8 > prio_len) __builtin_amdgcn_s_setprio(1);
        // kLog: this user's log segment, rows s .. s+n-1 (n * qrow < 2^30 bytes)
        const rsrc_t l_rs = LOG ? make_rsrc(qlog + s * ldq, (uint32_t)n * qrow) : q_rs;
        const int32_t *__restrict__ it = items + s;
        const T *__restrict__ rt = ratings + s;
        const rsrc_t p_rs = make_rsrc(pu + (int64_t)u * ldu, (uint32_t)K * sizeof(T));
        const rsrc_t b_rs = make_rsrc(bu + u, sizeof(T));

        vec p[G];
#pragma unroll
        for (int v = 0; v < G; ++v) p[v] = L::template ld<0>(p_rs, cu[v]) + one[v];
        T bu_u = Buf<T>::template ld<0>(b_rs, 0);
        const T sqrt_n = sqrt(T(n));  // mf.pyx:470
        const T rs_n = T(1) / sqrt_n;  // one division per user; the terms are multiplied

        // SVD++: walk the user's y_j rows: 64 item ids per vector load (lane l holds entry
        // x0 + l, read back with v_readlane), rows gathered kYB at a time; rows past the user's
        // list get an out-of-range offset (load 0, store / atomic dropped).
        constexpr int kYB = 32;
        auto walk_y = [&](auto &&consume) {
            for (int x0 = 0; x0 < n; x0 += kWave) {
                const int gid = it[x0 + lane < n ? x0 + lane : n - 1];
                const int cnt = n - x0 < kWave ? n - x0 : kWave;
                for (int x = 0; x < cnt; x += kYB) {
                    T g[kYB][U];
                    uint32_t ro[kYB];
#pragma unroll
                    for (int a = 0; a < kYB; ++a) {
                        ro[a] = (uint32_t)readlane(gid, x + a < kWave ? x + a : kWave - 1) * yrow +
                                (x + a < cnt ? 0u : y_oob);
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            g[a][u] = Buf<T>::template ld<kYLdAux>(y_rs, ro[a] + cy1[u]);
                    }
                    consume(g, ro);
                }
            }
        };
        // SVD++ (1): u_impl = sum_{j in I_u} y_j / sqrt|I_u|  (mf.pyx:473-476, per-term division)
        vec imp[G], imp0[G];
#pragma unroll
        for (int v = 0; v < G; ++v) imp[v] = L::splat(T(0));
        if (PP) {
            T imp1[U];
#pragma unroll
            for (int u = 0; u < U; ++u) imp1[u] = T(0);
            walk_y([&](T (&g)[kYB][U], uint32_t (&)[kYB]) {
#pragma unroll
                for (int a = 0; a < kYB; ++a)
#pragma unroll
                    for (int u = 0; u < U; ++u) imp1[u] += g[a][u] * rs_n;
            });
            to_lane8<G>(imp1, imp);
        }
#pragma unroll
        for (int v = 0; v < G; ++v) imp0[v] = imp[v];
        T A = T(1);

        // software pipeline: slot d holds the gathered row of rating j0 + d.  The item ids and
        // ratings of a group travel one group ahead in VGPR lanes (lane l < kPF holds entry l,
        // clamped to the user's last rating, so every gathered row is a real row), are loaded
        // once per group by two unconditional vector loads, and are read with v_readlane.
        auto grp_load = [&](int j0, int &gi, T &gr) {
            int j = j0 + (lane & (kPF - 1));
            j = j < n ? j : n - 1;
            gi = it[j];
            gr = rt[j];
        };
        int gi_b, gi_n;
        T gr_b, gr_n;
        uint32_t s_off[kPF];
        T s_r[kPF];
        vec s_q[kPF][G];
        {
            int gi_a;
            T gr_a;
            grp_load(0, gi_a, gr_a);
            grp_load(kPF, gi_b, gr_b);
            // both groups resolved here (group a is needed right away anyway): otherwise the
            // loop would inherit "group b may be in flight" from this path and wait for it with
            // a conservative, near-empty vmcnt at every iteration
            asm volatile("" ::"v"(gi_a), "v"(gr_a), "v"(gi_b), "v"(gr_b));  // (no sinking)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int d = 0; d < kPF; ++d) {
                s_off[d] = (uint32_t)readlane(gi_a, d) * qrow;
                s_r[d] = readlane(gr_a, d);
#pragma unroll
                for (int v = 0; v < G; ++v) s_q[d][v] = L::template lds<kLdAux>(q_rs, cq[v], s_off[d]);
                __builtin_amdgcn_sched_barrier(0);  // keep slot order: slot 0's row lands first
            }
        }
        // c = mu + bu is carried instead of bu: err = (r - c) - dot, and
        // c' = mu + bu' = lr_bu err + [(1 - lr_bu reg_bu) c + mu lr_bu reg_bu], the bracket off
        // the chain (bu = c - mu is stored at the end)
        T cb = hp.gm + bu_u;
        const T kb = hp.gm * (T(1) - abu);
        T cb_0 = abu * cb + kb;

        // One rating in slot d.  FULL: every slot of the group is a real rating and the slot is
        // refilled with rating j0 + kPF + d; tail group: slots past n run masked, no refill.
        auto step = [&](auto full_c, const int j0, const int d) {
            constexpr bool FULL = decltype(full_c)::value;
            const bool valid = FULL || j0 + d < n;
            vec pe[G], part2 = L::splat(T(0));
#pragma unroll
            for (int v = 0; v < G; ++v) {
                pe[v] = PP ? p[v] + imp[v] : p[v];
                part2 += s_q[d][v] * pe[v];
            }
            // everything that does not need err: fills the reduction's DPP wait states
            vec dq_e[G], dq_0[G], dp_e[G], dp_0[G], dy_e[G];
#pragma unroll
            for (int v = 0; v < G; ++v) {
                const vec q = s_q[d][v];
                dq_e[v] = lrq[v] * pe[v];  // d  = err (lr pe) + (-lr reg q)
                dq_0[v] = nrq[v] * q;
                dp_e[v] = lrp[v] * q;      // p' = err (lr q) + (1 - lr reg) p
                dp_0[v] = ap[v] * p[v];
                if (PP) dy_e[v] = lry[v] * q;
            }
            const T dot = wave_sum_u(L::hsum(part2));  // <q_i, p_u (+imp)> + b_i
            const T e0 = s_r[d] - cb;
            const T err = e0 - dot;                      // mf.pyx:250 / :483
            vec qd[G];
#pragma unroll
            for (int v = 0; v < G; ++v) {  // mf.pyx:258-262 / :490-498, old puf and qif
                // (kLog logs the gradient err pe; mf_log_apply applies lr and reg per column)
                qd[v] = LOG ? err * pe[v] : err * dq_e[v] + dq_0[v];
                const vec pn = err * dp_e[v] + dp_0[v];
                p[v] = valid ? pn : p[v];
                if (PP) {  // imp' = decay imp + lr_yj err q (the c of y_j <- A y_j + c: below)
                    const vec in = decay * imp[v] + err * dy_e[v];
                    imp[v] = valid ? in : imp[v];
                }
            }
            const T cbn = lr_bu * err + cb_0;  // mf.pyx:253-254
            cb = valid ? cbn : cb;
            cb_0 = abu * cb + kb;
            if (PP) A = valid ? A * decay : A;
            const uint32_t off = s_off[d];
            vec stv[G];  // the row after this rating (kPlain stores it; DUPS forwards it)
#pragma unroll
            for (int v = 0; v < G; ++v) stv[v] = s_q[d][v] + qd[v];
            T qd1[U];  // kAtomic: the delta in the Lane1 view (contiguous 256-B atomics)
            if (ATOM) to_lane1<G>(qd, qd1);
            if (FULL) {  // real rows only: the row offset rides in soffset, no address math
#pragma unroll
                for (int v = 0; v < G; ++v) {
                    if (LOG) L::template sts<0>(l_rs, cl[v], (uint32_t)(j0 + d) * qrow, qd[v]);
                    if (MODE == kPlain) L::template sts<0>(q_rs, cq[v], off, stv[v]);
                }
                if (ATOM)
#pragma unroll
                    for (int u = 0; u < U; ++u) atom_add1(q_rs, qb, q_oob, cq1[u], off, qd1[u]);
            } else {     // masked slots: push the offset past the table / log segment
                const uint32_t moff = valid ? off : off + q_oob;
#pragma unroll
                for (int v = 0; v < G; ++v) {
                    if (LOG) L::template st<0>(l_rs, (uint32_t)(j0 + d) * qrow + cl[v], qd[v]);
                    if (MODE == kPlain) L::template st<0>(q_rs, moff + cq[v], stv[v]);
                }
                if (ATOM)
#pragma unroll
                    for (int u = 0; u < U; ++u) atom_add1(q_rs, qb, q_oob, moff + cq1[u], 0, qd1[u]);
            }
            // keep the next gather below the last use of the slot's old row: hoisting it would
            // need a second register set and a copy (and a wait) at the loop latch
            __builtin_amdgcn_sched_barrier(0);
            if (FULL) {
                s_off[d] = (uint32_t)readlane(gi_b, d) * qrow;
                s_r[d] = readlane(gr_b, d);
#pragma unroll
                for (int v = 0; v < G; ++v) s_q[d][v] = L::template lds<kLdAux>(q_rs, cq[v], s_off[d]);
            }
            if (DUPS && valid) {  // same item again within the window: forward the row
#pragma unroll
                for (int dd = 0; dd < kPF; ++dd)
                    if (s_off[dd] == off)
#pragma unroll
                        for (int v = 0; v < G; ++v) s_q[dd][v] = stv[v];
            }
        };
        int j0 = 0;
        for (; j0 + kPF <= n; j0 += kPF) {
            grp_load(j0 + 2 * kPF, gi_n, gr_n);
#pragma unroll
            for (int d = 0; d < kPF; ++d) step(std::true_type{}, j0, d);
            gi_b = gi_n;
            gr_b = gr_n;
        }
        if (j0 < n) {
#pragma unroll
            for (int d = 0; d < kPF; ++d) step(std::false_type{}, j0, d);
        }
#pragma unroll
        for (int v = 0; v < G; ++v) L::template st<0>(p_rs, cu[v], p[v]);
        bu_u = cb - hp.gm;
        Buf<T>::template st<0>(b_rs, lane == 0 ? 0u : (uint32_t)sizeof(T), bu_u);
        __builtin_amdgcn_s_setprio(0);

        // SVD++ (3): y_j <- A y_j + c for every j in I_u
        if (PP) {
            // c obeys the same recurrence as imp (c' = decay c + lr_yj err q / sqrt n) from 0
            // instead of imp0, so c = (imp - A imp0) / sqrt n: no per-rating c update
            vec cacc[G];
#pragma unroll
            for (int v = 0; v < G; ++v) cacc[v] = (imp[v] - A * imp0[v]) * rs_n;
            if (ycbuf) {  // deferred: mf_svdpp_y_fold adds every user's c to its y_j after the chunk
                const rsrc_t c_rs = make_rsrc(ycbuf + (int64_t)u * ldu, (uint32_t)K * sizeof(T));
#pragma unroll
                for (int v = 0; v < G; ++v) L::template st<0>(c_rs, cu[v], cacc[v]);
                return;
            }
            T cacc1[U];
            to_lane1<G>(cacc, cacc1);
            walk_y([&](T (&g)[kYB][U], uint32_t (&ro)[kYB]) {
#pragma unroll
                for (int a = 0; a < kYB; ++a)
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (YATOM)
                            atom_add1(y_rs, yj, y_oob, cy1[u], ro[a], (A - T(1)) * g[a][u] + cacc1[u]);
                        else
                            Buf<T>::template st<0>(y_rs, ro[a] + cy1[u], A * g[a][u] + cacc1[u]);
                    }
            });
        }
    };

    for (int64_t w = wave; w < n_sched; w += n_waves) do_user(sched[w]);
}

// checkpoint interval of the SVD log (elog != NULL): one user row per pair of ratings (the
// replay's inverse step needs exactly 2)
constexpr int kCkpt = 2;
// The checkpoint rows are packed: pair m (ratings 2m, 2m + 1 of the user) of the user whose
// ratings start at CSR position s = row_ptr[u] is row ck_row0(s, u) + m.  ((s + u + 1) / 2 grows
// by >= ceil(n_u / 2) from one user to the next: no per-user table, at most one spare row per
// user; the log holds ck_row0(nnz, n_users) rows.)  Written rows are contiguous, so every cache
// line of a user's rows is written whole (row stride 2 left half-written lines between rows).
__host__ __device__ __forceinline__ int64_t ck_row0(int64_t s, int64_t u) { return (s + u + 1) >> 1; }
#ifndef MF_LA_MAX_G
#define MF_LA_MAX_G 2  // lookahead body / checkpoint log for rows of up to 2 lane groups (1 KiB)
#endif
constexpr int kLaMaxG = MF_LA_MAX_G;
#ifndef MF_LA_BANK_G2
#define MF_LA_BANK_G2 8  // the same for two lane groups per row
#endif
#ifndef MF_LA_BANK_SB
#define MF_LA_BANK_SB 16  // ... with the biases beside one lane group (SB: fp32 K=128)
#endif
#ifndef MF_LA_BANK
#define MF_LA_BANK 8  // ratings per bank in the lookahead body (two banks alternate)
#endif
#ifndef MF_LA_IDS_AHEAD
#define MF_LA_IDS_AHEAD 2  // the SVD lookahead body loads a bank's item ids this many banks ahead
#endif
#ifndef MF_LOG_AUX
#define MF_LOG_AUX 0  // cache policy of the lookahead body's log stores
#endif
#ifndef MF_STREAM_AUX
#define MF_STREAM_AUX 0  // epoch kernel: cache policy of the CSR reads and the user-row stream
#endif
#ifndef MF_ELOG_AUX
#define MF_ELOG_AUX 0  // epoch kernel: cache policy of the error-log stores
#endif

// ---- two 64-lane sums at once (the lookahead body's X and Y): the halves are exchanged with one
// v_permlane32_swap so that lanes 0-31 carry x's partials and lanes 32-63 y's, then one 5-step
// DPP reduction inside each half (the last step a row_bcast:15) leaves x's sum in lane 31 and
// y's in lane 63: 9 instructions for both (one wave_sum_u alone is 8).
__device__ __forceinline__ void swap32(float &a, float &b) {
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, a), __builtin_bit_cast(int, b),
                                              false, false);
    a = __builtin_bit_cast(float, (int)r[0]);
    b = __builtin_bit_cast(float, (int)r[1]);
}
__device__ __forceinline__ void swap32(double &a, double &b) {
    const long long ua = __builtin_bit_cast(long long, a), ub = __builtin_bit_cast(long long, b);
    float al = __builtin_bit_cast(float, (int)(ua & 0xffffffffll));
    float ah = __builtin_bit_cast(float, (int)(ua >> 32));
    float bl = __builtin_bit_cast(float, (int)(ub & 0xffffffffll));
    float bh = __builtin_bit_cast(float, (int)(ub >> 32));
    swap32(al, bl);
    swap32(ah, bh);
    auto join = [](float lo, float hi) {
        return __builtin_bit_cast(double, ((long long)__builtin_bit_cast(int, hi) << 32) |
                                              (unsigned int)__builtin_bit_cast(int, lo));
    };
    a = join(al, ah);
    b = join(bl, bh);
}
template <typename T>
__device__ __forceinline__ void wave_sum2_u(T x, T y, T &sx, T &sy) {
    swap32(x, y);     // x = [x_lo | y_lo], y = [x_hi | y_hi]
    T z = x + y;      // lanes 0-31: x's partials, lanes 32-63: y's
    z += dpp<0xB1>(z);   // quad_perm [1,0,3,2]
    z += dpp<0x4E>(z);   // quad_perm [2,3,0,1]
    z += dpp<0x141>(z);  // row_half_mirror
    z += dpp<0x140>(z);  // row_mirror: every row holds its 16-lane sum
    z += dpp<0x142>(z);  // row_bcast:15: row 1 += row 0, row 3 += row 2 (rows 0, 2: unused)
    sx = readlane(z, 31);
    sy = readlane(z, 63);
}

// ---- SVD rating loop in lookahead form (kLog, SVD, G = 1: K <= 127 fp32 / K <= 63 fp64)
//
// Per user, with q_k = the snapshot row [q | b] of rating k and p_k's column K the constant 1:
//   dot_k = <q_k, p_k>,  err_k = r_k - c_k - dot_k,  c_k = mu + bu_k,
//   p_{k+1} = ap o p_k + err_k D_k,  D_k = lrp o q_k   (ap = 1 - lr_pu reg_pu, lrp = lr_pu on
//   factor columns; 1 and 0 elsewhere),  c_{k+1} = lr_bu err_k + c0_k,  c0_k = abu c_k + kb.
// One step back, dot_k = X_k + err_{k-1} Y_k with X_k = <q_k, ap o p_{k-1}>, Y_k = <q_k, D_{k-1}>:
//   err_k = (r_k - c0_{k-1}) - X_k - err_{k-1} (Y_k + lr_bu)        -- one FMA after err_{k-1}.
// X_{k+1} and Y_{k+1} need p_k = A_{k-1} + err_{k-1} D_{k-1} (A = ap o p), i.e. err_{k-1}: their
// reduction (wave_sum2_u) runs a whole rating ahead of its use, beside the next rating's work,
// instead of on the err -> p -> dot -> err chain.  The log row of rating k is g_k = err_k p_k
// (columns 0..K; mf_log_apply turns the sums into the item steps).  Same arithmetic as the
// reference recursion up to rounding (fp64: equal to the delta-log oracle to 1e-9,
// tests/test_gpu_parity.py).
// The user bias rides in the row too: column K+1 of the user row holds c_k = mu + bu_k and the
// item table's column K+1 is the constant 1 (MF_MODE_LOG's layout, include/surprise_amd.h), with
// ap = abu, lrp = lr_bu and a constant kb added to A in that column: c's recursion
// c_{k+1} = abu c_k + kb + lr_bu err_k is the row's own, <q_k, p_k> includes c_k and Y_k includes
// lr_bu, so err_k = r_k - X_k - err_{k-1} Y_k with no scalar bias recursion beside it.
// SB (narrow checkpoint rows, K * size a multiple of 512 B: fp32 K=128): the lane groups cover
// the K factor columns only; the item bias b_k (column K) is loaded beside each row as a
// wave-uniform element and the user bias c_k = mu + bu_k is the scalar recursion
// c_{k+1} = C0_k + lr_bu err_k, C0_k = abu c_k + kb: X_{k+1} gains b_{k+1} + C0_k and Y_{k+1}
// gains lr_bu -- the same err_k as the in-row form, with one lane group instead of two.
template <typename T, int G, bool CK, bool ER = false, bool SB = false, bool NT = false>
__device__ __forceinline__ void epoch_body_la(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, int ldu, T *qb, int ldq, T *qlog, T *elog, int K,
    int biased, Hyper<T> hp, int n_items, int64_t n_waves_req, int xmask, double *psq,
    int err_col, int ck_ld, const T *__restrict__ ibias = nullptr)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    // ratings per bank of gathered rows (a power of 2 <= 64)
    // (SB -- narrow checkpoint rows, the C4 layout -- gathers its rows in banks of 16: the epoch
    // kernel at C4 19.7 -> 18.9 ms, profiles/r4q_bank_sweep.txt; banks of 4: 25.0)
    constexpr int kB = SB ? MF_LA_BANK_SB : (G == 1 ? MF_LA_BANK : MF_LA_BANK_G2);
    static_assert(!CK || (kB % kCkpt == 0 && kB <= kWave), "checkpoints: whole banks");
    constexpr int kAhead = MF_LA_IDS_AHEAD;  // banks between a bank's id loads and its gathers
    // the log stores' cache policy: NT (MF_EPOCH_LOG_NT) streams them past the caches
    constexpr int kLogAux = NT ? kNt : MF_LOG_AUX;
    static_assert(kAhead >= 2, "the next bank's ids are loaded before its rows");
    const int lane = threadIdx.x & (kWave - 1);
    int64_t wave, grid_waves;
    if (!wave_slot(xmask, wave, grid_waves)) return;
    SlotSettle settle(lane == 0 ? xmask : 0, wave, grid_waves, wave_grid_index());
    const int64_t n_waves = n_waves_req < grid_waves ? n_waves_req : grid_waves;
    if (wave >= n_waves) return;

    const uint32_t qrow = (uint32_t)ldq * sizeof(T), prow = (uint32_t)ldu * sizeof(T);
    const uint32_t q_oob = (uint32_t)n_items * qrow;
    // CK: the checkpoint rows' stride, ldq or (MF_EPOCH_CKPT_NARROW) K: the factor columns only
    const uint32_t lrow = CK ? (uint32_t)ck_ld * sizeof(T) : qrow;
    const int l_cols = ER ? err_col : (CK && ck_ld < ldq ? K : ldq);  // columns a log row stores
    const T lr_bu = biased ? hp.lr_bu : T(0);
    const T abu = T(1) - lr_bu * hp.reg_bu;
    const T kb = hp.gm * (T(1) - abu);
    const uint32_t kbo = (uint32_t)K * sizeof(T);  // SB: the item bias's offset in a row
    uint32_t cq[G], cu[G], cl[G];
    vec one[G], lrp[G], ap[G], kvec[G], cvec[G];
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;
        const uint32_t b = (uint32_t)c0 * sizeof(T);
        cq[v] = c0 < ldq ? b : q_oob;
        cu[v] = c0 < ldu ? b : prow;  // >= the pu record (K elements): dropped
        cl[v] = c0 < l_cols ? b : kLogOob;  // (ER: the err columns' own store)
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const int c = c0 + e;
            const bool fac = c < K, bias = biased && c == K, ub = c == K + 1;
            L::set(one[v], e, bias ? T(1) : T(0));
            L::set(cvec[v], e, ub ? T(1) : T(0));
            L::set(lrp[v], e, fac ? hp.lr_pu : (ub ? lr_bu : T(0)));
            L::set(ap[v], e, fac ? T(1) - hp.lr_pu * hp.reg_pu : (ub ? abu : T(1)));
            L::set(kvec[v], e, ub ? kb : T(0));
        }
    }
    // the lane and element of column K+1 (c = mu + bu)
    const int cb_lane = ((K + 1) / W) % kWave, cb_grp = ((K + 1) / W) / kWave, cb_e = (K + 1) % W;
    // err_col > 0: lane d < kB of a bank's err vector goes to its pair's checkpoint row (the
    // bank's row d / 2), column err_col + (d & 1)
    const uint32_t ce = (ER && lane < kB)
                            ? (uint32_t)(((lane >> 1) * ldq + err_col + (lane & 1)) * sizeof(T))
                            : kLogOob;
    const rsrc_t q_rs = make_rsrc(qb, q_oob);
    // SB with the item-bias mirror (the rsrc is only read where ibias is given)
    const rsrc_t ib_rs = make_rsrc(ibias, (uint32_t)n_items * sizeof(T));
    const int prio_len = (int)(row_ptr[sched[0] + 1] - row_ptr[sched[0]]);

    auto do_user = [&](const int u) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        if (n <= 0) return;
        if (n * 2 > prio_len) __builtin_amdgcn_s_setprio(3);
        else if (n * 4 > prio_len) __builtin_amdgcn_s_setprio(2);
        else if (n * 8 > prio_len) __builtin_amdgcn_s_setprio(1);
        // CK: the user's checkpoint rows, one per pair, packed (ck_row0); else row k per rating
        const rsrc_t l_rs = CK ? make_rsrc(qlog + ck_row0(s, u) * ck_ld, (uint32_t)((n + 1) / 2) * lrow)
                               : make_rsrc(qlog + s * ldq, (uint32_t)n * qrow);
        const rsrc_t e_rs = make_rsrc(CK && !ER ? elog + s : qlog, (uint32_t)n * sizeof(T));
        const int32_t *__restrict__ it = items + s;
        const T *__restrict__ rt = ratings + s;
        const rsrc_t p_rs = make_rsrc(pu + (int64_t)u * ldu, (uint32_t)K * sizeof(T));
        const rsrc_t b_rs = make_rsrc(bu + u, sizeof(T));

        // p_0 = [p_u | 1 | mu + bu]: the item bias's constant and the user bias in the row
        const T bu0 = Buf<T>::template ld<0>(b_rs, 0);
        vec p0[G];
#pragma unroll
        for (int v = 0; v < G; ++v)
            p0[v] = L::template ld<MF_STREAM_AUX>(p_rs, cu[v]) + one[v] + (hp.gm + bu0) * cvec[v];


        // Two banks of kB gathered rows alternate.  At the start of a bank: the ids of the bank
        // after next are requested, then the next bank's rows, THEN the previous bank's kB log
        // rows (held in registers) are stored.  vmcnt retires in issue order and a store stays
        // counted for thousands of cycles under load: this order lets every wait for a row skip
        // the most recent stores (a row's wait covers stores a whole bank older than it).
        // Rows past n are clamped to the user's last rating (real rows); their log stores fall
        // outside l_rs and are dropped.
        auto grp_load = [&](int j0, uint32_t &go, T &gr) {
            int j = j0 + (lane & (kB - 1));
            j = j < n ? j : n - 1;
            // (the item id itself: fill() scales it to the row offset, and the SB body with an
            // item-bias mirror indexes the mirror by it)
            if constexpr (MF_STREAM_AUX == kNt) {
                go = (uint32_t)__builtin_nontemporal_load(it + j);
                gr = __builtin_nontemporal_load(rt + j);
            } else {
                go = (uint32_t)it[j];
                gr = rt[j];
            }
        };
        vec bank[2][kB][G];
        T br[2][kB];
        T bbv[SB ? 2 : 1];  // SB: lane d holds the item bias of the bank's row d
        // log rows of the current bank: CK: per pair (c, c + 1) of the user's ratings (c even) the
        // row p_{c+1} at log row c, and err_k in lane k mod kB of ev; otherwise every rating's
        // gradient row g_k = err_k p_k
        constexpr int kLg = CK ? kB / kCkpt : kB;
        vec lg[kLg][G];
        T ev = T(0);
        // ids / ratings of the next kAhead - 1 banks (bank j0 + kB .. j0 + (kAhead - 1) kB), their
        // loads issued kAhead - 1 banks before the bank's row gathers need them
        uint32_t go_q[kAhead - 1];
        T gr_q[kAhead - 1];
        auto fill = [&](const int bk, const uint32_t go, const T gr) {
            // SB: the bank's item biases in ONE per-lane gather, issued before its rows (a wait
            // for them is not a wait for the rows): from the mirror -- an L2-resident array --
            // where one is given, so that a row gather touches only the row's factor lines (4
            // of 128 B at fp32 K=128 on 128-B rows instead of 5, profiles/r5u_probes.txt), else
            // from the rows' column K.  (Selecting between the two buffer resources instead of
            // branching miscompiled: every SB parity test failed, tools/runs/r5w_gpu.sh.)
            if constexpr (SB) {
                if (ibias)
                    bbv[bk] = Buf<T>::template ld<0>(ib_rs, go * (uint32_t)sizeof(T));
                else
                    bbv[bk] = Buf<T>::template ld<0>(q_rs, go * qrow + kbo);
            }
#pragma unroll
            for (int d = 0; d < kB; ++d) {
                const uint32_t gid = readlane((int)go, d);
                const uint32_t off = gid * qrow;
                br[bk][d] = readlane(gr, d);
#pragma unroll
                for (int v = 0; v < G; ++v) bank[bk][d][v] = L::template lds<0>(q_rs, cq[v], off);
            }
        };
        auto flush = [&](const int j0p) {  // log rows j0p .. j0p + kB - 1
            if constexpr (CK) {
#pragma unroll
                for (int x = 0; x < kLg; ++x)
#pragma unroll
                    for (int v = 0; v < G; ++v)
                        L::template sts<kLogAux>(l_rs, cl[v], (uint32_t)(j0p / kCkpt + x) * lrow,
                                                 lg[x][v]);
                // err_k: into its pair's row (columns err_col, err_col + 1; the row stores above
                // leave those columns alone) or to elog[k]; one store per bank either way
                if constexpr (ER)
                    Buf<T>::template st<0>(l_rs, ce + (uint32_t)(j0p / kCkpt) * lrow, ev);
                else
                    Buf<T>::template st<MF_ELOG_AUX>(e_rs, lane < kB ? (uint32_t)(j0p + lane) * sizeof(T) : kLogOob, ev);
                return;
            }
#pragma unroll
            for (int d = 0; d < kB; ++d) {
#pragma unroll
                for (int v = 0; v < G; ++v)
                    L::template sts<kLogAux>(l_rs, cl[v], (uint32_t)(j0p + d) * qrow, lg[d][v]);
            }
        };
        {
            uint32_t go0;
            T gr0;
            grp_load(0, go0, gr0);
#pragma unroll
            for (int a = 0; a < kAhead - 1; ++a) grp_load((a + 1) * kB, go_q[a], gr_q[a]);
            asm volatile("" ::"v"(go0), "v"(gr0), "v"(go_q[0]), "v"(gr_q[0]));
            __builtin_amdgcn_sched_barrier(0);
            fill(0, go0, gr0);
        }
        // state entering rating k: err_p = err_{k-1}, A_p = A_{k-1}, D_p = D_{k-1}, X = X_k,
        // Y = Y_k (k = 0: err_{-1} = 0, A_{-1} = p_0, D_{-1} = 0, X_0 = <q_0, p_0>)
        T err_p = T(0), X, Y = T(0);
        T C0_p = hp.gm + bu0;  // SB: C0_{k-1} (k = 0: c_0 itself, err_{-1} = 0)
        vec A_p[G], D_p[G];
        {
            vec part = L::splat(T(0));
#pragma unroll
            for (int v = 0; v < G; ++v) {
                A_p[v] = p0[v];
                D_p[v] = L::splat(T(0));
                part += bank[0][0][v] * p0[v];
            }
            X = wave_sum_u(L::hsum(part));
            if constexpr (SB) X += readlane(bbv[0], 0) + C0_p;
        }

        auto step = [&](auto full_c, auto bank_c, const int j0, const int d) {
            constexpr bool FULL = decltype(full_c)::value;
            constexpr int bk = decltype(bank_c)::value;
            const int k = j0 + d;
            const bool valid = FULL || k < n;
            vec (&qn)[G] = d + 1 < kB ? bank[bk][d + 1] : bank[bk ^ 1][0];  // rating k+1's row
            // keep the first read (and the wait) of rating k+1's row in this step, and the
            // steps' memory waits in order
#pragma unroll
            for (int v = 0; v < G; ++v) asm volatile("" : "+v"(qn[v])::"memory");
            // (X + err_p Y = <q_k, p_k> + c_k: the bias columns ride in the dot)
            const T err = (br[bk][d] - X) - err_p * Y;  // mf.pyx:250
            vec pk[G], A[G], D[G], px = L::splat(T(0)), py = L::splat(T(0));
#pragma unroll
            for (int v = 0; v < G; ++v) {
                // p_k, c_k (mf.pyx:253-262, one rating late)
                pk[v] = A_p[v] + err_p * D_p[v];
                A[v] = ap[v] * pk[v] + kvec[v];
                D[v] = lrp[v] * bank[bk][d][v];
                px += qn[v] * A[v];
                py += qn[v] * D[v];
                if (!CK) lg[d][v] = err * pk[v];  // the log row g_k = err_k p_k (old p, mf.pyx:261)
                // checkpoint of the pair (c, c + 1), c = k - 1 even: p_{c+1}, the row after
                // rating c (k = n: the user's final row, for odd n -- the masked tail step)
                else if (d % kCkpt == 1) lg[d / kCkpt][v] = pk[v];
            }
            if (CK) ev = lane == d ? err : ev;
            T Xn, Yn;
            wave_sum2_u(L::hsum(px), L::hsum(py), Xn, Yn);  // X_{k+1}, Y_{k+1}
            T C0 = T(0);
            if constexpr (SB) {  // c_k = C0_{k-1} + lr_bu err_{k-1}; C0_k = abu c_k + kb
                C0 = abu * (C0_p + lr_bu * err_p) + kb;
                const int bn = d + 1 < kB ? bk : bk ^ 1, dn = d + 1 < kB ? d + 1 : 0;
                Xn += readlane(bbv[bn], dn) + C0;
                Yn += lr_bu;
            }
            if (FULL) {
                err_p = err;
                X = Xn;
                Y = Yn;
                if constexpr (SB) C0_p = C0;
#pragma unroll
                for (int v = 0; v < G; ++v) {
                    A_p[v] = A[v];
                    D_p[v] = D[v];
                }
            } else {
                err_p = valid ? err : err_p;
                X = valid ? Xn : X;
                Y = valid ? Yn : Y;
                if constexpr (SB) C0_p = valid ? C0 : C0_p;
#pragma unroll
                for (int v = 0; v < G; ++v) {
                    A_p[v] = valid ? A[v] : A_p[v];
                    D_p[v] = valid ? D[v] : D_p[v];
                }
            }
        };
        int j0 = 0;
        // one full bank: ratings j0 .. j0 + kB - 1 in bank bk (FIRST: nothing to flush yet)
        auto full_bank = [&](auto bank_c, auto first_c) {
            constexpr int bk = decltype(bank_c)::value;
            uint32_t go_new;
            T gr_new;
            grp_load(j0 + kAhead * kB, go_new, gr_new);
            asm volatile("" ::: "memory");  // issue order: ids, rows, then the stores
            fill(bk ^ 1, go_q[0], gr_q[0]);
            asm volatile("" ::: "memory");
            if (!decltype(first_c)::value) flush(j0 - kB);
#pragma unroll
            for (int a = 0; a + 1 < kAhead - 1; ++a) {
                go_q[a] = go_q[a + 1];
                gr_q[a] = gr_q[a + 1];
            }
            go_q[kAhead - 2] = go_new;
            gr_q[kAhead - 2] = gr_new;
#pragma unroll
            for (int d = 0; d < kB; ++d) step(std::true_type{}, bank_c, j0, d);
            j0 += kB;
        };
        // the last ratings j0 .. n-1 (0 < n - j0 < kB) in bank bk: the previous bank's log rows
        // go out first (the steps reuse their registers), then masked steps and their rows
        auto tail_bank = [&](auto bank_c) {
            if (j0 > 0) flush(j0 - kB);
#pragma unroll
            for (int d = 0; d < kB; ++d) step(std::false_type{}, bank_c, j0, d);
            flush(j0);
        };
        using B0 = std::integral_constant<int, 0>;
        using B1 = std::integral_constant<int, 1>;
        using Yes = std::true_type;
        using No = std::false_type;
        if (n >= kB) {
            full_bank(B0{}, Yes{});
            while (j0 + 2 * kB <= n) {  // (full_bank advances j0)
                full_bank(B1{}, No{});
                full_bank(B0{}, No{});
            }
            if (j0 + kB <= n) {
                full_bank(B1{}, No{});
                if (j0 < n) tail_bank(B0{});
                else flush(j0 - kB);
            } else if (j0 < n) {
                tail_bank(B1{});
            } else {
                flush(j0 - kB);
            }
        } else {
            tail_bank(B0{});
        }
        // after rating n-1: p_n = A_{n-1} + err_{n-1} D_{n-1} (column K+1: c_n = mu + bu)
        double sq = 0;  // psq: sum of p_n^2 over the factor columns (the log fold's <p^2>)
        T cn = T(0);
#pragma unroll
        for (int v = 0; v < G; ++v) {
            const vec pn = A_p[v] + err_p * D_p[v];
            L::template st<MF_STREAM_AUX>(p_rs, cu[v], pn);
            if (!SB && v == cb_grp) cn = readlane(L::get(pn, cb_e), cb_lane);
#pragma unroll
            for (int e = 0; e < W; ++e) {
                const double x = (double)L::get(pn, e);
                sq += (lane + kWave * v) * W + e < K ? x * x : 0.0;
            }
        }
        if constexpr (SB) cn = C0_p + lr_bu * err_p;  // c_n
        if (psq) {
            sq = wave_sum(sq);
            if (lane == 0) psq[u] = sq;
        }
        const T bu_u = cn - hp.gm;
        Buf<T>::template st<0>(b_rs, lane == 0 ? 0u : (uint32_t)sizeof(T), bu_u);
        __builtin_amdgcn_s_setprio(0);
    };

    for (int64_t w = wave; w < n_sched; w += n_waves) {
        const int u = sched[w];
        if (u >= 0) do_user(u);  // (chain schedules are padded with -1)
    }
}

#ifndef MF_PP_LA
#define MF_PP_LA 1  // SVD++ (atomic q rows, deferred y): the lookahead body below
#endif

// ---- SVD++ q deltas through an LDS ring (MF_SVDPP_HELPERS): one chain wave per workgroup
// trains users; its per-rating q deltas go into a ring of row images in LDS and the workgroup's
// three other waves issue the float atomics.  A wave that issues float atomics itself is held
// by them (each stays counted in vmcnt for thousands of cycles and a wave can keep only a few
// dozen in flight): measured, the SVD++ epoch with the atomics in the chain wave took 2.4x the
// same loop without them.  Slot t % R holds rating t's delta row, written as the chain's 8-byte
// lane elements (a row image: byte c * sizeof(T) = column c) and read back one column per lane
// (64 consecutive dwords per atomic instruction).  head / tail[h]: ratings pushed / passed.
#ifndef MF_PP_HX_BANK
#define MF_PP_HX_BANK 8  // ratings per bank of gathered item rows in the helper-wave chain
#endif
#ifndef MF_PP_HX_BANK_G2
#define MF_PP_HX_BANK_G2 4  // ... with two lane groups (fp32 K > 126): 2 workgroups fit a CU
#endif
template <int G>
constexpr int hx_bank() { return G == 1 ? MF_PP_HX_BANK : MF_PP_HX_BANK_G2; }
constexpr int kHxHelpers = 3;  // helper waves per chain (MF_EPOCH_SVDPP_ONE_HELPER: 1)
constexpr int kSpinMax = 1 << 22;  // bounded spins (s_sleep 2 each, ~0.2 s): never hang the GPU
// MF_HX_SPIN_TEST (a test build, tests/test_gpu_ext.py): bits of the status word set by the caller
// before the launch make the bounded waits give up at once -- 0x100 the helpers' wait for rows,
// 0x200 the chain's wait for ring room -- so the failure paths run on purpose
#ifdef MF_HX_SPIN_TEST
constexpr int32_t kSpinTestHelper = 0x100, kSpinTestChain = 0x200;
__device__ __forceinline__ int spin_bound(const int32_t *status, int32_t bit) {
    return status && (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)
               ? 0 : kSpinMax;
}
#else
constexpr int32_t kSpinTestHelper = 0, kSpinTestChain = 0;
__device__ __forceinline__ int spin_bound(const int32_t *, int32_t) { return kSpinMax; }
#endif

template <typename T, int G, int H = kHxHelpers>
struct PPRing {
    static constexpr int R = 4 * hx_bank<G>();  // ring slots
    typename Lane8<T>::vec data[R][G][kWave];
    uint32_t off[R];
    T bias[R];  // SB: the slot's item-bias delta (the row's column K, outside the lane groups)
    int head, done;
    int tail[H];  // one per helper wave
};

// ring hand-off: the count is stored with release and read with acquire (workgroup scope: on
// gfx950 an s_waitcnt lgkmcnt(0) around the LDS access, no vmcnt wait), so the slots' rows are
// ordered before / after it by the memory model, not by the hardware's LDS ordering alone
__device__ __forceinline__ int lds_load(int *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// hx status word bits (mf_svdpp_epoch's status): a helper timed out waiting for rows (it exits;
// rows later pushed for it are lost: the chunk's item rows are invalid) / a chain found no room
// in the ring within the bound and issued that bank's atomics itself (results intact)
constexpr int32_t kHxHelperTimeout = MF_HX_HELPER_TIMEOUT, kHxChainFallback = MF_HX_CHAIN_FALLBACK;
__device__ __forceinline__ void set_status(int32_t *status, int32_t bit) {
    if (status && (threadIdx.x & (kWave - 1)) == 0)  // (a vector atomic, written through)
        __hip_atomic_fetch_or(status, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// helper wave h of a chain's H: issue the atomics of the slots t = h (mod H)
// (n_rows: the rows the slots' offsets may address -- 2 n_items with hot-row replicas;
// SB: each slot also carries the item-bias delta of column K, added by lane 0)
// MIX (the hybrid launch): a slot whose offset has bit 31 set is a cold item's gradient row,
// stored (plain stores) to row (off & 0x7FFFFFFF) / row size of the cold log clog instead
constexpr uint32_t kColdSlot = 0x80000000u;
template <typename T, int G, bool SB, int H, bool MIX = false>
__device__ void pp_ring_helper(PPRing<T, G, H> *ring, int h, T *qb, int ldq, int n_rows,
                               int32_t *status, int K = 0, T *clog = nullptr)
{
    constexpr int R = PPRing<T, G, H>::R;
    constexpr int U = Lane1<T, G>::U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t qrow = (uint32_t)ldq * sizeof(T), q_oob = (uint32_t)n_rows * qrow;
    const rsrc_t q_rs = make_rsrc(qb, q_oob);
    uint32_t cq1[U], cq1m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = lane + kWave * u;
        cq1[u] = c < ldq ? (uint32_t)c * sizeof(T) : q_oob;
        cq1m[u] = c < ldq ? (uint32_t)c * sizeof(T) : 0x7FFFF000u;  // (MIX: past the log)
    }
    const rsrc_t c_rs = make_rsrc(MIX ? (const void *)clog : (const void *)qb, 0x7FFFF000u);
    const T *img = (const T *)&ring->data[0][0][0];
    constexpr int kSlotT = G * kWave * (int)(sizeof(typename Lane8<T>::vec) / sizeof(T));
    const int spin_max = spin_bound(status, kSpinTestHelper);
    int t = 0, spins = 0;
    while (true) {
        int hd = lds_load(&ring->head);
        if (t >= hd) {
            if (lds_load(&ring->done)) {
                asm volatile("" ::: "memory");
                hd = lds_load(&ring->head);
                if (t >= hd) break;
            } else {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > spin_max) {  // (never hang the GPU: report and stop)
                    set_status(status, kHxHelperTimeout);
                    break;
                }
                continue;
            }
        }
        spins = 0;
        asm volatile("" ::: "memory");
        for (int tt = t + ((h - t % H) + H) % H; tt < hd; tt += H) {
            const int slot = tt % R;
            const uint32_t off = __builtin_amdgcn_readfirstlane(ring->off[slot]);
            T v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = img[slot * kSlotT + lane + kWave * u];
            if constexpr (MIX) {
                if (off & kColdSlot) {  // (a uniform branch)
                    const uint32_t lo = off & ~kColdSlot;
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        Buf<T>::template sts<0>(c_rs, cq1m[u], lo, v[u]);
                    if constexpr (SB)
                        Buf<T>::template sts<0>(c_rs, lane == 0 ? (uint32_t)K * sizeof(T)
                                                                : 0x7FFFF000u, lo, ring->bias[slot]);
                    continue;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) atom_add1(q_rs, qb, q_oob, cq1[u], off, v[u]);
            if constexpr (SB)  // (one lane: the other lanes' offset is past the table)
                atom_add1(q_rs, qb, q_oob, lane == 0 ? (uint32_t)K * sizeof(T) : q_oob, off,
                          ring->bias[slot]);
        }
        t = hd;
        lds_store(&ring->tail[h], t);  // (release: the slots' reads before the count)
    }
}

// ---- SVD++ rating loop in lookahead form (kAtomic, deferred y, G <= 2, no repeated items)
//
// SVDpp.sgd per rating (mf.pyx:478-498) in the exact per-user affine form: with m_k = u_impl
// before rating k (m_0 = sum_{j in I_u} y_j / sqrt|I_u|, one gather at the user's start) and
// s_k = p_k + m_k (column K: the constant 1 of the bias),
//   err_k = r_k - c_k - <q_k, s_k>,  p_{k+1} = ap o p_k + err_k lrp o q_k,
//   m_{k+1} = dc o m_k + err_k lry o q_k  (dc = 1 - lr_yj reg_yj, lry = lr_yj: every y_j of the
//   user takes the same step, so u_impl moves by lr_yj err q_k),
//   q_k += err_k lrq o s_k + nrq o q_k  (float atomics on the shared row, bias in column K).
// One rating back, s_k = B_{k-1} + err_{k-1} D_{k-1} with B = ap o p + dc o m and
// D = (lrp + lry) o q, so err_k = (r_k - c0_{k-1}) - X_k - err_{k-1} (Y_k + lr_bu) with
// X_k = <q_k, B_{k-1}>, Y_k = <q_k, D_{k-1}>: the recursion of epoch_body_la, whose reductions run
// a rating ahead of their use.  The q atomics of a bank are issued one bank late, after the next
// bank's row gathers (a row's vmcnt wait then never covers an atomic younger than a whole bank:
// an atomic stays counted for thousands of cycles under load).  The y update is deferred:
// c_u = (m_n - dc^n m_0) / sqrt|I_u| goes to ycbuf (mf_svdpp_y_fold applies it after the chunk).
//
// Hot-row replicas (HOT, the helper-wave launch): the float atomics on one row are performed one
// after the other at the memory side, so the most-rated items' rows bound the launch (C3: the
// top item's 4525 ratings of an epoch, ~0.12 us each).  An item with hot[i] != 0 has a delta
// replica at row n_items + i of qb: the chains of odd workgroups add its deltas there, the
// others to the row itself, and every read of the row adds the replica (the value one row would
// hold: no staleness added); mf_svdpp_hot_fold folds the replicas back after the chunk.
//
// q log (LQ, mf_svdpp_epoch_qlog): the item rows are a read-only chunk-start snapshot; each
// rating's q / b gradient g_k = err_k [s_k | 1] is stored (plain stores) as row urow[u] + k of the
// chunk's log instead of being added to the row, and mf_log_reduce / mf_log_apply fold the log
// after the chunk with the recency weights, as the SVD gradient log (oracle:
// oracle_svdpp_sgd_stalelog with every item stale).  No float atomic, no helper wave.
template <typename T, int G, bool HX, bool HOT = false, bool SB = false, int H = kHxHelpers,
          bool LQ = false, bool NT = false, bool SS = false, bool MIX = false>
__device__ __forceinline__ void epoch_body_pp_la(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, int ldu, T *qb, int ldq, T *yj, T *ycbuf, int K,
    Hyper<T> hp, int n_items, int64_t n_waves_req, int xmask, PPRing<T, G, H> *ring,
    int32_t *status, const uint8_t *__restrict__ hot = nullptr, T *qlog = nullptr,
    const int64_t *__restrict__ urow = nullptr, double *__restrict__ psq = nullptr,
    const int32_t *__restrict__ crow = nullptr)
{
    static_assert(!(LQ && (HX || HOT)), "the q log: no helper waves, no hot replicas");
    // MIX (the helper-wave launch, mf_svdpp_epoch_mix): the cold items' rows stay read-only for
    // the chunk -- their ratings' q / b gradients go to the item-grouped log (row crow[p] of
    // qlog, folded after the chunk like the q log's) -- and only the other items' deltas go to
    // the helper waves' float atomics (oracle_svdpp_sgd_stalelog with the cold items stale)
    static_assert(!MIX || (HX && !LQ), "the hybrid launch: helper waves, no q log");
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    // (the chain of a helper-wave launch is alone on its SIMD: registers for deeper banks)
    constexpr int kB = HX ? hx_bank<G>() : (G == 1 ? MF_LA_BANK : MF_LA_BANK_G2);
    constexpr int U = Lane1<T, G>::U;
    const int lane = threadIdx.x & (kWave - 1);
    int64_t wave, grid_waves;
    if (HX) {  // one chain per workgroup (wave 0; the others are pp_ring_helper)
        wave = blockIdx.x;
        grid_waves = gridDim.x;
    } else if (!wave_slot(xmask, wave, grid_waves)) {
        return;
    }
    SlotSettle settle(!HX && lane == 0 ? xmask : 0, wave, grid_waves, wave_grid_index());
    const int64_t n_waves = n_waves_req < grid_waves ? n_waves_req : grid_waves;
    if (wave >= n_waves) return;

    const uint32_t qrow = (uint32_t)ldq * sizeof(T), yrow = (uint32_t)ldu * sizeof(T);
    // (HOT: the table's range covers the replicas, rows n_items .. 2 n_items - 1)
    const uint32_t rep_shift = (uint32_t)n_items * qrow;
    const uint32_t q_oob = (HOT ? 2u : 1u) * rep_shift, y_oob = (uint32_t)n_items * yrow;
    const bool to_rep = HOT && (blockIdx.x & 1);  // this chain's hot deltas: to the replicas
    // SB (the lane groups cover the K factor columns only, K * size a multiple of 512 B): the item
    // bias, column K, rides beside the row as one wave-uniform element per rating
    const uint32_t kbo = (uint32_t)K * sizeof(T);
    int pushed = 0;  // HX: ratings pushed to the ring
    const int chain_spins = HX ? spin_bound(status, kSpinTestChain) : 0;
    uint32_t cq[G], cu[G], cq1[U], cy1[U], cqm[MIX ? G : 1];
    vec one[G], lrp[G], ap[G], lry[G], lrpy[G], lrq[G], nrq[G];
    const T dc = T(1) - hp.lr_yj * hp.reg_yj;
    // a lane past the row: its column offset is past the item table AND past any user's log
    // segment (< 2^30 bytes) -- both ranges dropped (voffset + soffset, no 32-bit wrap)
    constexpr uint32_t kColOob = 0x7FFFF000u;
    const uint32_t col_oob = LQ ? kColOob : q_oob;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = lane + kWave * u;
        cq1[u] = c < ldq ? (uint32_t)c * sizeof(T) : q_oob;
        cy1[u] = c < ldu ? (uint32_t)c * sizeof(T) : y_oob;
    }
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;
        const uint32_t b = (uint32_t)c0 * sizeof(T);
        cq[v] = c0 < ldq ? b : col_oob;
        if constexpr (MIX) cqm[v] = c0 < ldq ? b : kColOob;  // (the cold log's: past its range)
        cu[v] = c0 < ldu ? b : y_oob;  // >= the pu / ycbuf records (K elements) too: dropped
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const int c = c0 + e;
            const bool fac = c < K, bias = c == K;
            const T lq = fac ? hp.lr_qi : (bias ? hp.lr_bi : T(0));
            const T rq = fac ? hp.reg_qi : (bias ? hp.reg_bi : T(0));
            L::set(one[v], e, bias ? T(1) : T(0));
            L::set(lrp[v], e, fac ? hp.lr_pu : T(0));
            L::set(ap[v], e, fac ? T(1) - hp.lr_pu * hp.reg_pu : T(1));
            L::set(lry[v], e, fac ? hp.lr_yj : T(0));
            L::set(lrpy[v], e, fac ? hp.lr_pu + hp.lr_yj : T(0));
            L::set(lrq[v], e, lq);
            L::set(nrq[v], e, -lq * rq);
        }
    }
    const T lr_bu = hp.lr_bu;
    const T abu = T(1) - lr_bu * hp.reg_bu;
    const T kb = hp.gm * (T(1) - abu);
    const rsrc_t q_rs = make_rsrc(qb, q_oob);
    const rsrc_t y_rs = make_rsrc(yj, y_oob);
    // MIX: the cold log (rows crow[p] of qlog; a masked row's offset lies past kMaxTable)
    const rsrc_t c_rs = make_rsrc(MIX ? (const void *)qlog : (const void *)qb, 0x7FFFF000u);
    const int prio_len = (int)(row_ptr[sched[0] + 1] - row_ptr[sched[0]]);

    auto do_user = [&](const int u) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        if (n <= 0) return;
        if (n * 2 > prio_len) __builtin_amdgcn_s_setprio(3);
        else if (n * 4 > prio_len) __builtin_amdgcn_s_setprio(2);
        else if (n * 8 > prio_len) __builtin_amdgcn_s_setprio(1);
        const int32_t *__restrict__ it = items + s;
        const T *__restrict__ rt = ratings + s;
        const int32_t *__restrict__ cw = crow + (MIX ? s : 0);
        const rsrc_t p_rs = make_rsrc(pu + (int64_t)u * ldu, (uint32_t)K * sizeof(T));
        const rsrc_t b_rs = make_rsrc(bu + u, sizeof(T));
        // LQ: the user's rows of the chunk's log (row k = its k-th rating)
        const rsrc_t l_rs = LQ ? make_rsrc(qlog + urow[u] * ldq, (uint32_t)n * qrow) : q_rs;
        const T rs_n = T(1) / sqrt(T(n));  // mf.pyx:470-476

        vec p0[G];
#pragma unroll
        for (int v = 0; v < G; ++v) p0[v] = L::template ld<0>(p_rs, cu[v]) + one[v];
        const T bu0 = Buf<T>::template ld<0>(b_rs, 0);

        // u_impl at the user's start: the y_j rows (chunk-start values: the fold is deferred)
        // gathered 32 at a time in the Lane1 view, 64 item ids per vector load
        vec m0[G];
        {
            constexpr int kYB = 32;
            T acc1[U];
#pragma unroll
            for (int uu = 0; uu < U; ++uu) acc1[uu] = T(0);
            for (int x0 = 0; x0 < n; x0 += kWave) {
                const int gid = it[x0 + lane < n ? x0 + lane : n - 1];
                const int cnt = n - x0 < kWave ? n - x0 : kWave;
                for (int x = 0; x < cnt; x += kYB) {
                    T g[kYB][U];
#pragma unroll
                    for (int a = 0; a < kYB; ++a) {
                        const uint32_t ro = (uint32_t)readlane(gid, x + a < kWave ? x + a : kWave - 1) *
                                                yrow + (x + a < cnt ? 0u : y_oob);
#pragma unroll
                        for (int uu = 0; uu < U; ++uu) g[a][uu] = Buf<T>::template ld<0>(y_rs, ro + cy1[uu]);
                    }
#pragma unroll
                    for (int a = 0; a < kYB; ++a)
#pragma unroll
                        for (int uu = 0; uu < U; ++uu) acc1[uu] += g[a][uu] * rs_n;
                }
            }
            to_lane8<G>(acc1, m0);
        }

        auto grp_load = [&](int j0, uint32_t &go, T &gr, int &gh) {
            int j = j0 + (lane & (kB - 1));
            j = j < n ? j : n - 1;
            const int i = it[j];
            go = (uint32_t)i * qrow;
            gr = rt[j];
            if constexpr (HOT) gh = hot[i];
            // MIX: gh < 0 marks a cold item's rating, its log row -gh - 1 (a cold item is never
            // a hot-replica item: those are the most-rated)
            if constexpr (MIX) {
                if constexpr (!HOT) gh = 0;  // (gh is the caller's variable: no stale value)
                const int c = cw[j];
                if (c >= 0) gh = -c - 1;
            }
        };
        vec bank[2][kB][G];
        T bbv[SB ? 2 : 1];  // SB: lane d holds the item bias of the bank's entry d
        vec rep[HOT ? 2 : 1][HOT ? kB : 1][G];  // HOT: the replica rows of a bank's entries
        int cr[MIX ? 2 : 1][MIX ? kB : 1];  // MIX: entry d's cold log row, or -1
        uint32_t cbits = 0;  // MIX: bit d = entry d of the bank being flushed went to the log
        T br[2][kB];
        uint32_t bo[2][kB];
        uint32_t hm[2] = {0u, 0u};  // HOT: bit d = entry d of the bank is a hot item
        vec dl[kB][G];      // the q deltas of the current bank (issued one bank late)
        T dlb[SB ? kB : 1];  // SB: their item-bias deltas
        uint32_t dlo[kB];   // their row offsets (masked ratings: past the table)
        uint32_t go_n1, go_n2;
        T gr_n1, gr_n2;
        int gh_n1 = 0, gh_n2 = 0;
        auto fill = [&](const int bk, const uint32_t go, const T gr, const int gh) {
            if constexpr (HOT)
                hm[bk] = (uint32_t)__builtin_amdgcn_ballot_w64(gh > 0) & ((1u << kB) - 1u);
            // SB: the bank's item biases in one per-lane gather before its rows (epoch_body_la)
            if constexpr (SB) bbv[bk] = Buf<T>::template ld<kSc1>(q_rs, go + kbo);
#pragma unroll
            for (int d = 0; d < kB; ++d) {
                const uint32_t off = readlane((int)go, d);
                bo[bk][d] = off;
                br[bk][d] = readlane(gr, d);
                if constexpr (MIX) {
                    const int g = readlane(gh, d);
                    cr[bk][d] = g < 0 ? -g - 1 : -1;
                }
#pragma unroll
                for (int v = 0; v < G; ++v) bank[bk][d][v] = L::template lds<kSc1>(q_rs, cq[v], off);
                if constexpr (HOT) {  // (a uniform branch: most entries are not hot)
                    if ((hm[bk] >> d) & 1u) {
#pragma unroll
                        for (int v = 0; v < G; ++v)
                            rep[bk][d][v] = L::template lds<kSc1>(q_rs, cq[v], off + rep_shift);
                    }
                }
            }
        };
        auto atomics = [&]() {  // the previous bank's q deltas as float atomics, from this wave
#pragma unroll
            for (int d = 0; d < kB; ++d) {
                if (MIX && ((cbits >> d) & 1u)) {  // (a cold entry: its row to the log)
#pragma unroll
                    for (int v = 0; v < G; ++v) L::template sts<0>(c_rs, cqm[v], dlo[d], dl[d][v]);
                    if constexpr (SB)
                        Buf<T>::template sts<0>(c_rs, lane == 0 ? kbo : kColOob, dlo[d], dlb[d]);
                    continue;
                }
                T d1[U];
                to_lane1<G>(dl[d], d1);
#pragma unroll
                for (int uu = 0; uu < U; ++uu) atom_add1(q_rs, qb, q_oob, cq1[uu], dlo[d], d1[uu]);
                if constexpr (SB)
                    atom_add1(q_rs, qb, q_oob, lane == 0 ? kbo : q_oob, dlo[d], dlb[d]);
            }
        };
        auto flush = [&]() {  // the float atomics of the previous bank's ratings
            if constexpr (LQ) {  // ... or (the q log) the bank's gradient rows, plain stores
#pragma unroll
                for (int d = 0; d < kB; ++d) {
#pragma unroll
                    for (int v = 0; v < G; ++v)
                        L::template sts<NT ? kNt : 0>(l_rs, cq[v], dlo[d], dl[d][v]);
                    if constexpr (SB)
                        Buf<T>::template sts<NT ? kNt : 0>(l_rs, lane == 0 ? kbo : kColOob, dlo[d],
                                                           dlb[d]);
                }
                return;
            }
            if constexpr (HX) {  // ... handed to the helper waves through the ring
                constexpr int R = PPRing<T, G, H>::R;
                bool room = false;
                for (int spins = 0; spins < chain_spins; ++spins) {  // room for kB rows
                    int m = lds_load(&ring->tail[0]);
#pragma unroll
                    for (int h = 1; h < H; ++h) {
                        const int th = lds_load(&ring->tail[h]);
                        m = th < m ? th : m;
                    }
                    if (pushed + kB - m <= R) {
                        room = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (!room) {  // (no unconsumed slot is ever overwritten: this bank's atomics here)
                    set_status(status, kHxChainFallback);
                    atomics();
                    return;
                }
#pragma unroll
                for (int d = 0; d < kB; ++d) {
                    const int slot = (pushed + d) % R;
#pragma unroll
                    for (int v = 0; v < G; ++v) ring->data[slot][v][lane] = dl[d][v];
                    // (MIX: a cold entry's row goes to the log -- the helper stores it)
                    ring->off[slot] = MIX && ((cbits >> d) & 1u) ? dlo[d] | kColdSlot : dlo[d];
                    if constexpr (SB) ring->bias[slot] = dlb[d];
                }
                pushed += kB;
                lds_store(&ring->head, pushed);  // (release: the rows before the count)
            } else {
                atomics();
            }
        };
        {
            uint32_t go0;
            T gr0;
            int gh0 = 0;
            grp_load(0, go0, gr0, gh0);
            grp_load(kB, go_n1, gr_n1, gh_n1);
            asm volatile("" ::"v"(go0), "v"(gr0), "v"(go_n1), "v"(gr_n1));
            __builtin_amdgcn_sched_barrier(0);
            fill(0, go0, gr0, gh0);
        }
        // a bank entry's item row as the model sees it (HOT: + its replica)
        auto qrow_of = [&](const int bk, const int d, const int v) -> vec {
            if constexpr (HOT) {
                if ((hm[bk] >> d) & 1u) return bank[bk][d][v] + rep[bk][d][v];
            }
            return bank[bk][d][v];
        };
        // state entering rating k: err_p = err_{k-1}, c0_p = c0_{k-1}, Pp = ap o p_{k-1},
        // Mp = dc o m_{k-1}, Dpp = lrp o q_{k-1}, Dmp = lry o q_{k-1}, X = X_k, Yb = Y_k + lr_bu
        // (k = 0: err_{-1} = 0, c0_{-1} = c_0, Pp = p_0, Mp = m_0, X_0 = <q_0, p_0 + m_0>)
        T err_p = T(0), c0_p = hp.gm + bu0, X, Yb = T(0);
        // SS (lr_pu = lr_yj and reg_pu = reg_yj, the defaults): p and m take the same step, so
        // only s = p + m is carried -- Pp holds a o s_{k-1}, Dpp (lrp + lry) o q_{k-1} -- and
        // p - m decays as a^k (p_0 - m_0) with no data in it: p_n, m_n come back at the end.
        // Half the chain's vector work per rating, and four fewer row-sized registers.
        vec Pp[G], Mp[SS ? 1 : G], Dpp[G], Dmp[SS ? 1 : G];
        {
            vec part = L::splat(T(0));
#pragma unroll
            for (int v = 0; v < G; ++v) {
                if constexpr (SS) {
                    Pp[v] = p0[v] + m0[v];
                } else {
                    Pp[v] = p0[v];
                    Mp[v] = m0[v];
                    Dmp[v] = L::splat(T(0));
                }
                Dpp[v] = L::splat(T(0));
                part += qrow_of(0, 0, v) * (p0[v] + m0[v]);
            }
            X = wave_sum_u(L::hsum(part));
            if constexpr (SB) X += readlane(bbv[0], 0);
        }
        auto step = [&](auto full_c, auto bank_c, const int j0, const int d) {
            constexpr bool FULL = decltype(full_c)::value;
            constexpr int bk = decltype(bank_c)::value;
            const int k = j0 + d;
            const bool valid = FULL || k < n;
            const int bn = d + 1 < kB ? bk : bk ^ 1, dn = d + 1 < kB ? d + 1 : 0;
            vec qn[G];
#pragma unroll
            for (int v = 0; v < G; ++v) {
                asm volatile("" : "+v"(bank[bn][dn][v])::"memory");
                if constexpr (HOT) asm volatile("" : "+v"(rep[bn][dn][v])::"memory");
                qn[v] = qrow_of(bn, dn, v);
            }
            const T err = (br[bk][d] - c0_p) - X - err_p * Yb;  // mf.pyx:483
            const bool cold = MIX && valid && cr[bk][d] >= 0;  // (MIX: a cold item's rating)
            const T c0 = abu * (lr_bu * err_p + c0_p) + kb;     // mf.pyx:486, one rating late
            vec P[G], M[SS ? 1 : G], Dp[G], Dm[SS ? 1 : G], px = L::splat(T(0)),
                py = L::splat(T(0));
#pragma unroll
            for (int v = 0; v < G; ++v) {
                const vec q = qrow_of(bk, d, v);
                vec sk;
                if constexpr (SS) {  // s_k = a o s_{k-1} + err_{k-1} (lrp + lry) o q_{k-1}
                    sk = Pp[v] + err_p * Dpp[v];
                    P[v] = ap[v] * sk;
                    Dp[v] = lrpy[v] * q;
                    px += qn[v] * P[v];
                    py += qn[v] * Dp[v];
                } else {
                    const vec pk = Pp[v] + err_p * Dpp[v];  // p_k, m_k (one rating late)
                    const vec mk = Mp[v] + err_p * Dmp[v];
                    sk = pk + mk;                           // puf + u_impl (mf.pyx:491-493)
                    P[v] = ap[v] * pk;
                    M[v] = dc * mk;
                    Dp[v] = lrp[v] * q;
                    Dm[v] = lry[v] * q;
                    px += qn[v] * (P[v] + M[v]);
                    py += qn[v] * (lrpy[v] * q);
                }
                if constexpr (LQ) dl[d][v] = err * sk;  // the gradient (the fold applies lr, reg)
                else if (MIX && cold) dl[d][v] = err * sk;  // (a cold item: its gradient, logged)
                else dl[d][v] = err * (lrq[v] * sk) + nrq[v] * q;  // mf.pyx:489, :492
            }
            if constexpr (SB) {
                if (LQ || (MIX && cold)) dlb[d] = err;
                else dlb[d] = hp.lr_bi * (err - hp.reg_bi * readlane(bbv[bk], d));  // mf.pyx:489
            }
            const bool hot_d = HOT && to_rep && ((hm[bk] >> d) & 1u);
            if constexpr (LQ)  // (past the user's segment: dropped)
                dlo[d] = (uint32_t)(valid ? k : n) * qrow;
            else if (MIX && cold)
                dlo[d] = (uint32_t)cr[bk][d] * qrow;
            else
                dlo[d] = valid ? (hot_d ? bo[bk][d] + rep_shift : bo[bk][d]) : bo[bk][d] + q_oob;
            if constexpr (MIX) cbits = cold ? (cbits | (1u << d)) : (cbits & ~(1u << d));
            T Xn, Yn;
            wave_sum2_u(L::hsum(px), L::hsum(py), Xn, Yn);  // X_{k+1}, Y_{k+1}
            if constexpr (SB) Xn += readlane(bbv[bn], dn);  // (the next item's bias: s_k's column K is 1)
            err_p = valid ? err : err_p;
            c0_p = valid ? c0 : c0_p;
            X = valid ? Xn : X;
            Yb = valid ? Yn + lr_bu : Yb;
#pragma unroll
            for (int v = 0; v < G; ++v) {
                Pp[v] = valid ? P[v] : Pp[v];
                Dpp[v] = valid ? Dp[v] : Dpp[v];
                if constexpr (!SS) {
                    Mp[v] = valid ? M[v] : Mp[v];
                    Dmp[v] = valid ? Dm[v] : Dmp[v];
                }
            }
        };
        int j0 = 0;
        auto full_bank = [&](auto bank_c, auto first_c) {
            constexpr int bk = decltype(bank_c)::value;
            grp_load(j0 + 2 * kB, go_n2, gr_n2, gh_n2);
            asm volatile("" ::: "memory");  // issue order: ids, rows, then the atomics
            fill(bk ^ 1, go_n1, gr_n1, gh_n1);
            asm volatile("" ::: "memory");
            if (!decltype(first_c)::value) flush();
            go_n1 = go_n2;
            gr_n1 = gr_n2;
            gh_n1 = gh_n2;
#pragma unroll
            for (int d = 0; d < kB; ++d) step(std::true_type{}, bank_c, j0, d);
            j0 += kB;
        };
        auto tail_bank = [&](auto bank_c) {
            if (j0 > 0) flush();
#pragma unroll
            for (int d = 0; d < kB; ++d) step(std::false_type{}, bank_c, j0, d);
            flush();
        };
        using B0 = std::integral_constant<int, 0>;
        using B1 = std::integral_constant<int, 1>;
        if (n >= kB) {
            full_bank(B0{}, std::true_type{});
            while (j0 + 2 * kB <= n) {
                full_bank(B1{}, std::false_type{});
                full_bank(B0{}, std::false_type{});
            }
            if (j0 + kB <= n) {
                full_bank(B1{}, std::false_type{});
                if (j0 < n) tail_bank(B0{});
                else flush();
            } else if (j0 < n) {
                tail_bank(B1{});
            } else {
                flush();
            }
        } else {
            tail_bank(B0{});
        }
        // after rating n-1: p_n, m_n (u_impl), c_n
        vec cacc[G];
        const T A = pow_int(dc, n);
        double sq = 0;  // LQ with psq: |p_n|^2 over the factor columns (the fold's <p^2>)
#pragma unroll
        for (int v = 0; v < G; ++v) {
            vec pn, mn;
            if constexpr (SS) {  // p_n - m_n = a^n (p_0 - m_0) (column K: 1, both ways)
                const vec sn = Pp[v] + err_p * Dpp[v];
                const vec dn = A * (p0[v] - m0[v]) + (T(1) - A) * one[v];
                pn = T(0.5) * (sn + dn);
                mn = T(0.5) * (sn - dn);
            } else {
                pn = Pp[v] + err_p * Dpp[v];
                mn = Mp[v] + err_p * Dmp[v];
            }
            L::template st<0>(p_rs, cu[v], pn);
            cacc[v] = (mn - A * m0[v]) * rs_n;
            if constexpr (LQ || MIX) {
#pragma unroll
                for (int e = 0; e < W; ++e) {
                    const double x = (double)L::get(pn, e);
                    sq += (lane + kWave * v) * W + e < K ? x * x : 0.0;
                }
            }
        }
        if ((LQ || MIX) && psq) {
            sq = wave_sum(sq);
            if (lane == 0) psq[u] = sq;
        }
        const T bu_u = lr_bu * err_p + c0_p - hp.gm;
        Buf<T>::template st<0>(b_rs, lane == 0 ? 0u : (uint32_t)sizeof(T), bu_u);
        const rsrc_t c_rs = make_rsrc(ycbuf + (int64_t)u * ldu, (uint32_t)K * sizeof(T));
#pragma unroll
        for (int v = 0; v < G; ++v) L::template st<0>(c_rs, cu[v], cacc[v]);
        __builtin_amdgcn_s_setprio(0);
    };

    for (int64_t w = wave; w < n_sched; w += n_waves) {
        const int u = sched[w];
        if (u >= 0) do_user(u);  // (HX schedules are padded with -1)
    }
    if constexpr (HX) lds_store(&ring->done, 1);
}

#ifndef MF_LA
#define MF_LA 1
#endif

#define MF_EPOCH_PARAMS                                                                       \
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,                      \
        const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,       \
        T *__restrict__ pu, T *__restrict__ bu, int ldu, T *qb, int ldq, T *yj, T *qlog, T *elog,\
        int K, int biased, Hyper<T> hp, int n_items, int64_t n_waves_req, int xmask, double *psq,   \
        int err_col, int ck_ld
#define MF_EPOCH_ARGS \
    row_ptr, items, ratings, sched, n_sched, pu, bu, ldu, qb, ldq, yj, qlog, elog, K, biased, hp,    \
        n_items, n_waves_req, xmask

template <typename T, int G, int MODE, bool PP, bool DUPS>
__global__ __launch_bounds__(kBlock) void mf_epoch_kernel(MF_EPOCH_PARAMS)
{
    if constexpr (MODE == kAtomic && PP && !DUPS && G <= kLaMaxG && MF_PP_LA) {
        if (elog) {  // deferred y (elog = ycbuf)
            epoch_body_pp_la<T, G, false>(row_ptr, items, ratings, sched, n_sched, pu, bu, ldu,
                                          qb, ldq, yj, elog, K, hp, n_items, n_waves_req, xmask,
                                          (PPRing<T, G> *)nullptr, nullptr);
            return;
        }
    }
    if constexpr (MODE == kLog && !PP && G <= kLaMaxG && MF_LA) {  // (the gradient log)
        epoch_body_la<T, G, false>(row_ptr, items, ratings, sched, n_sched, pu, bu, ldu, qb, ldq,
                                   qlog, elog, K, biased, hp, n_items, n_waves_req, xmask, psq, 0,
                                   ldq);
    } else {
        epoch_body<T, G, MODE, PP, DUPS, kPF>(MF_EPOCH_ARGS);
    }
}

// SVD checkpoint log (elog != NULL): its own kernel, so that its register allocation is its own
// (ER: the errors go into the checkpoint rows, MF_EPOCH_ERR_IN_ROW; SB: the biases beside the
// lane groups, narrow rows of whole groups)
template <typename T, int G, bool ER, bool SB = false, bool NT = false>
__global__ __launch_bounds__(kBlock) void mf_ckpt_epoch_kernel(MF_EPOCH_PARAMS)
{
    // (yj: SVD has none -- the slot carries the SB body's item-bias mirror, nullable)
    epoch_body_la<T, G, true, ER, SB, NT>(row_ptr, items, ratings, sched, n_sched, pu, bu, ldu, qb,
                                      ldq, qlog, elog, K, biased, hp, n_items, n_waves_req, xmask,
                                      psq, err_col, ck_ld, (const T *)yj);
}

// SVD++ with helper waves (MF_SVDPP_HELPERS): workgroup = chain wave 0 + H atomic waves (3, or 1
// with MF_EPOCH_SVDPP_ONE_HELPER: a workgroup of two waves, twice the chains per CU in the same
// registers; a helper keeps up with a chain as long as its ~2 atomics per rating stay below the
// few dozen a wave keeps in flight for ~3000 cycles each)
// SB: the lane groups cover the K factor columns only and the item bias (column K) is carried as
// a scalar per rating (fp32 K=128: one lane group instead of two -- half the vector work and the
// registers of a bank of 8 rows)
template <typename T, int G, bool HOT, bool SB = false, int H = kHxHelpers, bool SS = false,
          bool MIX = false>
__global__ __launch_bounds__(kWave * (1 + H)) void mf_svdpp_hx_kernel(MF_EPOCH_PARAMS,
                                                                     int32_t *status,
                                                                     const uint8_t *hot,
                                                                     const int32_t *crow)
{
    __shared__ PPRing<T, G, H> ring;
    const int w = threadIdx.x / kWave;
    if (threadIdx.x == 0) {
        ring.head = 0;
        ring.done = 0;
        for (int h = 0; h < H; ++h) ring.tail[h] = 0;
    }
    __syncthreads();
    if (w == 0) {
        epoch_body_pp_la<T, G, true, HOT, SB, H, false, false, SS, MIX>(
            row_ptr, items, ratings, sched, n_sched, pu, bu, ldu, qb, ldq, yj, elog, K, hp,
            n_items, n_waves_req, 0, &ring, status, hot, qlog, nullptr, psq, crow);
        if (blockIdx.x >= n_waves_req) lds_store(&ring.done, 1);  // (no chain in this workgroup)
    } else {
        pp_ring_helper<T, G, SB, H, MIX>(&ring, w - 1, qb, ldq, (HOT ? 2 : 1) * n_items, status,
                                         K, qlog);
    }
}

// SVD++ with the q log (mf_svdpp_epoch_qlog): every wave a user chain, the item rows read-only,
// each rating's gradient row stored to the chunk's log (urow[u]: the user's first log row)
template <typename T, int G, bool SB, bool NT = false, bool SS = false>
__global__ __launch_bounds__(kBlock) void mf_svdpp_qlog_kernel(MF_EPOCH_PARAMS,
                                                              const int64_t *urow)
{
    epoch_body_pp_la<T, G, false, false, SB, 1, true, NT, SS>(
        row_ptr, items, ratings, sched, n_sched, pu, bu, ldu, qb, ldq, yj, elog, K, hp, n_items,
        n_waves_req, xmask, (PPRing<T, G, 1> *)nullptr, nullptr, nullptr, qlog, urow, psq);
}

}  // namespace

#ifdef MF_TU_EPOCH
namespace mf_ext {
template <typename T, int M, bool PP>
int launch_epoch_tm(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                    int32_t ldu, void *qb, int32_t ldq, void *yj, void *qlog, void *elog, int32_t K,
                    int32_t biased, const mf_hyper_t *hp, int64_t waves, bool dups, int xmask,
                    int hx, double *psq, int err_col, int ck_ld, int32_t *status,
                    const uint8_t *hot, const int64_t *urow, bool nt, const int32_t *crow,
                    void *stream)
{
    if ((psq || err_col) && (PP || M != kLog || !elog) && !(psq && (urow || crow) && !err_col))
        return set_err(MF_E_UNSUPPORTED, "user_sq / errors in rows: the SVD checkpoint log, the SVD++ q log or the hybrid launch only");
    // the lookahead body (SVD, MF_MODE_LOG, rows <= 1 KiB) carries the user bias in column K + 1
    if (!PP && M == kLog && MF_LA && (int64_t)ldq * sizeof(T) <= 512 * kLaMaxG && ldq < K + 2)
        return set_err(MF_E_ARG, "MF_MODE_LOG: ldq >= n_factors + 2 (the user-bias column)");
    // the factor columns fill whole lane groups and the bias column alone would need another
    const bool whole = ((int64_t)K * sizeof(T)) % 512 == 0 &&
                       (int64_t)K * sizeof(T) < ((int64_t)ldq * sizeof(T) + 511) / 512 * 512;
    // elog: SVD: the checkpoint log (the lookahead body: kLog, up to two lane groups -- of the
    //       whole row, or with narrow rows of whole groups (the biases beside the groups, SB) of
    //       the factor columns: fp64 K = 128, rows of 1088 B);
    //       SVD++: the deferred y buffer (kAtomic)
    const bool sb_rows = ck_ld < ldq && err_col <= 0 && whole &&
                         (int64_t)K * sizeof(T) <= 512 * kLaMaxG;
    if (elog && !PP && (M != kLog || !MF_LA || ((int64_t)ldq * sizeof(T) > 512 * kLaMaxG && !sb_rows)))
        return set_err(MF_E_UNSUPPORTED, "checkpoint log: SVD, MF_MODE_LOG, ldq * size <= 1 KiB "
                                         "(or narrow rows of whole lane groups) only");
    // (with the kLog snapshot the error stays stale for the whole chunk and the undamped sum of a
    // popular item's c_u diverges: measured held-out RMSE 1.82 on ML-1M)
    // ... unless the q log's chunks are small (mf_svdpp_epoch_qlog: urow given)
    if (elog && PP && !(M == kAtomic || (M == kLog && urow)))
        return set_err(MF_E_UNSUPPORTED, "deferred y: MF_MODE_ATOMIC, or the q log");
    if (urow && !(PP && M == kLog && elog && qlog && !dups && !hx && !hot))
        return set_err(MF_E_UNSUPPORTED, "the q log: SVD++, deferred y, no repeated items");
    if (hx && !(PP && M == kAtomic && elog && !dups))
        return set_err(MF_E_UNSUPPORTED, "helper waves: SVD++, MF_MODE_ATOMIC, deferred y, no repeated items");
    if (hot && !hx) return set_err(MF_E_ARG, "hot-row replicas: the helper-wave launch only");
    if (crow && !(hx && qlog && psq))
        return set_err(MF_E_UNSUPPORTED, "the hybrid launch: helper waves, a cold log, user_sq");
    // the helper-wave launch with the item bias beside the lane groups (SB) where the factor
    // columns fill whole groups
    const bool sb = hx && !hot && whole;
    // ... and the SVD checkpoint epoch with narrow rows (the rows hold the factor columns only)
    const bool sbk = !PP && M == kLog && elog && sb_rows;
    // SVD++: p and m take the same step where lr_pu = lr_yj and reg_pu = reg_yj (the reference's
    // defaults, lr_all / reg_all): the shared-step chain (epoch_body_pp_la SS)
    const bool ss = PP && hp->lr_pu == hp->lr_yj && hp->reg_pu == hp->reg_yj;
    return dispatch_g<T>(sb || sbk || (urow && whole) ? K : ldq, [&](auto gc) -> int {
        constexpr int V = decltype(gc)::value;
        if constexpr (PP && M == kAtomic && V <= kLaMaxG) {
            if (hx) {  // one workgroup per chain: wave 0 trains, waves 1..hx issue the q atomics
                // (ss: p and m share their step -- the shared-step chain of epoch_body_pp_la)
                auto kern = hx == 1 ? (hot ? (ss ? mf_svdpp_hx_kernel<T, V, true, false, 1, true>
                                                 : mf_svdpp_hx_kernel<T, V, true, false, 1>)
                                       : sb  ? (ss ? mf_svdpp_hx_kernel<T, V, false, true, 1, true>
                                                   : mf_svdpp_hx_kernel<T, V, false, true, 1>)
                                             : (ss ? mf_svdpp_hx_kernel<T, V, false, false, 1, true>
                                                   : mf_svdpp_hx_kernel<T, V, false, false, 1>))
                          : hot ? (ss ? mf_svdpp_hx_kernel<T, V, true, false, kHxHelpers, true>
                                      : mf_svdpp_hx_kernel<T, V, true>)
                          : sb  ? (ss ? mf_svdpp_hx_kernel<T, V, false, true, kHxHelpers, true>
                                      : mf_svdpp_hx_kernel<T, V, false, true>)
                                : (ss ? mf_svdpp_hx_kernel<T, V, false, false, kHxHelpers, true>
                                      : mf_svdpp_hx_kernel<T, V, false>);
                if (crow) {  // the hybrid launch (MIX): three helpers, any hot / SB layout
                    kern = hot ? (ss ? mf_svdpp_hx_kernel<T, V, true, false, kHxHelpers, true, true>
                                     : mf_svdpp_hx_kernel<T, V, true, false, kHxHelpers, false, true>)
                         : sb  ? (ss ? mf_svdpp_hx_kernel<T, V, false, true, kHxHelpers, true, true>
                                     : mf_svdpp_hx_kernel<T, V, false, true, kHxHelpers, false, true>)
                               : (ss ? mf_svdpp_hx_kernel<T, V, false, false, kHxHelpers, true, true>
                                     : mf_svdpp_hx_kernel<T, V, false, false, kHxHelpers, false, true>);
                    if (hx != kHxHelpers)
                        return set_err(MF_E_UNSUPPORTED, "the hybrid launch: three helper waves");
                }
                hipLaunchKernelGGL(kern, dim3(waves), dim3(kWave * (1 + hx)), 0,
                                   (hipStream_t)stream, csr->row_ptr, csr->items,
                                   (const T *)csr->ratings, sched, n_sched, (T *)pu, (T *)bu, ldu,
                                   (T *)qb, ldq, (T *)yj, (T *)qlog, (T *)elog, K, biased,
                                   cast_hyper<T>(hp), csr->n_items, waves, 0, psq, 0, ldq,
                                   status, hot, crow);
                return check_launch("mf_svdpp_hx_kernel");
            }
        } else {
            if (hx) return set_err(MF_E_UNSUPPORTED, "helper waves: rows of <= 1 KiB");
        }
        if constexpr (PP && M == kLog && V <= kLaMaxG) {
            if (urow) {  // the q log: a user chain per wave, gradient rows to the chunk's log
                auto kern = whole ? (nt ? (ss ? mf_svdpp_qlog_kernel<T, V, true, true, true>
                                              : mf_svdpp_qlog_kernel<T, V, true, true>)
                                        : (ss ? mf_svdpp_qlog_kernel<T, V, true, false, true>
                                              : mf_svdpp_qlog_kernel<T, V, true>))
                                  : (nt ? (ss ? mf_svdpp_qlog_kernel<T, V, false, true, true>
                                              : mf_svdpp_qlog_kernel<T, V, false, true>)
                                        : (ss ? mf_svdpp_qlog_kernel<T, V, false, false, true>
                                              : mf_svdpp_qlog_kernel<T, V, false>));
                hipLaunchKernelGGL(kern, dim3(grid_for_waves_x(waves, xmask)), dim3(kBlock), 0,
                                   (hipStream_t)stream, csr->row_ptr, csr->items,
                                   (const T *)csr->ratings, sched, n_sched, (T *)pu, (T *)bu, ldu,
                                   (T *)qb, ldq, (T *)yj, (T *)qlog, (T *)elog, K, biased,
                                   cast_hyper<T>(hp), csr->n_items, waves, xmask, psq, 0, ldq,
                                   urow);
                return check_launch("mf_svdpp_qlog_kernel");
            }
        } else {
            if (urow) return set_err(MF_E_UNSUPPORTED, "the q log: rows of <= 1 KiB");
        }
        if constexpr (M == kLog && !PP && V <= kLaMaxG && MF_LA) {
            if (elog) {  // the checkpoint log
                auto ck = err_col > 0 ? (nt ? mf_ckpt_epoch_kernel<T, V, true, false, true>
                                            : mf_ckpt_epoch_kernel<T, V, true>)
                          : sbk ? (nt ? mf_ckpt_epoch_kernel<T, V, false, true, true>
                                      : mf_ckpt_epoch_kernel<T, V, false, true>)
                                : (nt ? mf_ckpt_epoch_kernel<T, V, false, false, true>
                                      : mf_ckpt_epoch_kernel<T, V, false>);
                hipLaunchKernelGGL(ck, dim3(grid_for_waves_x(waves, xmask)), dim3(kBlock), 0,
                                   (hipStream_t)stream, csr->row_ptr, csr->items,
                                   (const T *)csr->ratings, sched, n_sched, (T *)pu, (T *)bu, ldu,
                                   (T *)qb, ldq, (T *)yj, (T *)qlog, (T *)elog, K, biased,
                                   cast_hyper<T>(hp), csr->n_items, waves, xmask, psq, err_col,
                                   ck_ld);
                return check_launch("mf_ckpt_epoch_kernel");
            }
        }
        // (kLog reads a snapshot: a repeated item sees the chunk-start row, no forwarding)
        auto kern = (dups && M != kLog) ? mf_epoch_kernel<T, V, M, PP, true>
                                        : mf_epoch_kernel<T, V, M, PP, false>;
        hipLaunchKernelGGL(kern, dim3(grid_for_waves_x(waves, xmask)), dim3(kBlock), 0,
                           (hipStream_t)stream,
                           csr->row_ptr, csr->items, (const T *)csr->ratings, sched, n_sched,
                           (T *)pu, (T *)bu, ldu, (T *)qb, ldq, (T *)yj, (T *)qlog, (T *)elog, K,
                           biased, cast_hyper<T>(hp), csr->n_items, waves, xmask, psq, err_col,
                           ldq);
        return check_launch(PP ? "mf_epoch_kernel<svdpp>" : "mf_epoch_kernel<svd>");
    });
}
template int launch_epoch_tm<MF_INST_T, MF_INST_M, (bool)MF_INST_PP>(
    const mf_csr_t *, const int32_t *, int64_t, void *, void *, int32_t, void *, int32_t, void *,
    void *, void *, int32_t, int32_t, const mf_hyper_t *, int64_t, bool, int, int, double *,
    int, int, int32_t *, const uint8_t *, const int64_t *, bool, const int32_t *, void *);
template <typename T, int M, bool PP>
int dispatch_sum_tm(unsigned long long *out)
{
    return dispatch_sum_here(out);
}
template int dispatch_sum_tm<MF_INST_T, MF_INST_M, (bool)MF_INST_PP>(unsigned long long *);
}  // namespace mf_ext
#else  // the main translation unit

namespace mf_ext {
thread_local char g_err[256] = "";
// mf_launch_event: the event the next mf_log_apply / mf_log_replay launch of this thread signals
thread_local hipEvent_t g_stop_event = nullptr;
// mf_launch_join: the join role of the next mf_log_replay launch of this thread
struct JoinArgs {
    uint32_t *words = nullptr;
    int role = 0;
    uint32_t epoch = 0;
};
thread_local JoinArgs g_join;
JoinArgs take_join() {
    const JoinArgs j = g_join;
    g_join = JoinArgs{};
    return j;
}
// mf_launch_fold: the fold inside the next mf_log_replay launch of this thread (cnt == NULL: off)
struct FoldArgs {
    void *qb = nullptr;
    const int32_t *ipp_a = nullptr, *ipp_b = nullptr;  // per item: its pieces in sums_a / sums_b
    const void *sums_a = nullptr, *sums_b = nullptr;
    const int32_t *totals = nullptr;
    int32_t *cnt = nullptr;    // per item: its pieces completed so far (0 between folds)
    uint32_t *blk = nullptr;   // the launches' block-arrival counters (MF_FOLD_WORDS)
    const double *p2stat = nullptr;
    double *stat_next = nullptr;
    const double *user_sq = nullptr;
    void *bias_out = nullptr;
    int64_t n_users = 0;
    int ld = 0, n_fac = 0, bias_col = -1, count_rule = 0, role = 0, n_launch = 0;
    double eta_b = 0, lr_c = 0, reg_c = 0, lr_f = 0, reg_f = 0, lr_b = 0, reg_b = 0;
};
thread_local FoldArgs g_fold;
FoldArgs take_fold() {
    const FoldArgs f = g_fold;
    g_fold = FoldArgs{};
    return f;
}
}

namespace {


// ---------------------------------------------------------------- hot-row replicas (SVD++)
// row i += replica row n_items + i, replica = 0, for the listed items (mf_svdpp_hot_fold)
template <typename T>
__global__ __launch_bounds__(kBlock) void hot_fold_kernel(T *qb, int ldq, int n_items,
                                                          const int32_t *__restrict__ hot_items,
                                                          int64_t total)
{
    for (int64_t x = blockIdx.x * (int64_t)kBlock + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * kBlock) {
        const int64_t i = hot_items[x / ldq], c = x % ldq;
        T *rep = qb + (n_items + i) * ldq + c;
        qb[i * ldq + c] += *rep;
        *rep = T(0);
    }
}

// ---------------------------------------------------------------- item-table merge (epoch-chunk)
//
// After an epoch-chunk, copy r of an item table (one per rank) holds snapshot + d_r.  Plain SUM of the d_r
// is right while every replica made only a few small steps on a row, and overshoots by up to a
// factor n_replicas once the steps saturate (a popular item's bias converges within one chunk
// in every replica).  The count-aware merge weights each replica's delta per row by
//     w_r = (n_r / N) (1 - (1-eta)^N) / (1 - (1-eta)^{n_r}),    N = sum_r n_r  (all ranks),
// the exact combination for a scalar SGD recursion x <- x + eta (t - x) with n_r steps per
// replica: -> 1 (SUM) while eta N << 1, -> n_r / N (count-weighted MEAN) when saturated.
// eta per column: lr_bi (1 + reg_bi) for the bias column, lr_qi (<p^2> + reg_qi) for factor
// columns (<p^2> = mean squared user factor, measured on the device at merge time).

template <typename T>
__global__ __launch_bounds__(kBlock) void sumsq_kernel(const T *__restrict__ x, int64_t n_rows,
                                                       int K, int ld, double *out)
{
    __shared__ double part[kBlock / kWave];
    double acc = 0;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    // 4 rows' loads in flight per wave (a row is 1-2 loads per lane: latency-bound otherwise)
    constexpr int kR = 4;
    for (int64_t r0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave; r0 < n_rows;
         r0 += kR * n_waves)
        for (int c = lane; c < K; c += kWave) {
            T v[kR];
#pragma unroll
            for (int y = 0; y < kR; ++y) {
                const int64_t r = r0 + y * n_waves;
                v[y] = r < n_rows ? x[r * ld + c] : T(0);
            }
#pragma unroll
            for (int y = 0; y < kR; ++y) acc += (double)v[y] * (double)v[y];
        }
    acc = wave_sum(acc);
    if ((threadIdx.x & (kWave - 1)) == 0) part[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int w = 0; w < kBlock / kWave; ++w) t += part[w];
        atomicAdd(out, t);
        if (blockIdx.x == 0) atomicAdd(out + 1, (double)n_rows * K);  // {sum, count}
    }
}

// sum of sq[0..n) in a fixed order by one whole workgroup (per-thread strided sums, 32 loads in
// flight, then a fixed tree in LDS); the result in thread 0.  COH: loads at the agent's coherence
// point (sq written by another launch still running beside this one: the replay's fold)
template <bool COH = false>
__device__ __forceinline__ double block_sum(const double *__restrict__ sq, int64_t n)
{
    __shared__ double part[kBlock];
    double acc = 0;
    constexpr int kU = 32;  // loads in flight per thread (the sum order does not depend on it)
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)kU * kBlock) {
        double v[kU];
#pragma unroll
        for (int a = 0; a < kU; ++a) {
            const int64_t i = i0 + (int64_t)a * kBlock;
            if constexpr (COH)
                v[a] = i < n ? __hip_atomic_load(sq + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0.0;
            else
                v[a] = i < n ? sq[i] : 0.0;
        }
#pragma unroll
        for (int a = 0; a < kU; ++a) acc += v[a];
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
        __syncthreads();
    }
    return part[0];
}

// The <p^2> statistic {sum of sq[0..n), n * K} for the next chunk.  Up to kSqPartsMin users one
// workgroup sums them (fixed order).  Above it -- one workgroup's ~32 GB/s made the sum the tail
// of every C5 fold (10M users: 80 MB, ~2.5 ms per chunk) -- user_sq_parts_kernel, launched just
// before on the same stream, has left kSqParts fixed-range partial sums in out[2 ..], and thread
// 0 adds them in order.  Either way bit-reproducible.
constexpr int kSqParts = MF_SQ_PARTS;
constexpr int64_t kSqPartsMin = MF_SQ_PARTS_MIN;
template <bool COH = false>
__device__ __forceinline__ void block_sum_sq(const double *__restrict__ sq, int64_t n, int K,
                                             double *out)
{
    if (n >= kSqPartsMin) {
        if (threadIdx.x == 0) {
            double t = 0;
            for (int b = 0; b < kSqParts; ++b) t += out[2 + b];
            out[0] = t;
            out[1] = (double)n * K;
        }
        return;
    }
    const double t = block_sum<COH>(sq, n);
    if (threadIdx.x == 0) {
        out[0] = t;
        out[1] = (double)n * K;
    }
}

// block b: the sum of sq over [n b / P, n (b + 1) / P) in a fixed order -> parts[b]
__global__ __launch_bounds__(kBlock) void user_sq_parts_kernel(const double *__restrict__ sq,
                                                               int64_t n, double *__restrict__ parts)
{
    const int64_t lo = n * blockIdx.x / kSqParts, hi = n * (blockIdx.x + 1) / kSqParts;
    const double t = block_sum(sq + lo, hi - lo);
    if (threadIdx.x == 0) parts[blockIdx.x] = t;
}

// the partial sums block_sum_sq reads above kSqPartsMin users (stat: 2 + kSqParts doubles)
static int launch_sq_parts(const double *sq, int64_t n, double *stat, hipStream_t st)
{
    if (!sq || !stat || n < kSqPartsMin) return 0;
    hipLaunchKernelGGL(user_sq_parts_kernel, dim3(kSqParts), dim3(kBlock), 0, st, sq, n, stat + 2);
    return check_launch("user_sq_parts_kernel");
}

// Per-user sum of squares of the factor columns (fp64), one wave per row: the initial values of
// the user_sq array that the checkpoint-log epoch (mf_svd_epoch_sq) keeps current.
template <typename T>
__global__ __launch_bounds__(kBlock) void user_sq_kernel(const T *__restrict__ x, int64_t n_rows,
                                                         int K, int ld, double *__restrict__ out)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t r = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave; r < n_rows; r += n_waves) {
        double acc = 0;
        for (int c = lane; c < K; c += kWave) {
            const double v = (double)x[r * ld + c];
            acc += v * v;
        }
        acc = wave_sum(acc);
        if (lane == 0) out[r] = acc;
    }
}

// {sum of user_sq[0..n), n * K} in a fixed order (one block: strided per-thread sums, then a
// fixed tree): the <p^2> statistic of the log fold, bit-reproducible
__global__ __launch_bounds__(kBlock) void user_sq_reduce_kernel(const double *__restrict__ sq,
                                                                int64_t n, int K, double *out)
{
    block_sum_sq(sq, n, K, out);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void item_merge_kernel(
    T *tab, T *snap, int n_items, int ld, int n_fac, int bias_col, int n_rep,
    const int32_t *__restrict__ counts, const int32_t *__restrict__ totals, int rule,
    double l1m_bias, double lr_fac, double reg_fac, const double *__restrict__ p2stat,
    T *__restrict__ delta, int apply)
{
    const int64_t total = (int64_t)n_items * ld, stride = total;
    const bool mean = rule == MF_MERGE_MEAN, rec = rule == MF_MERGE_RECENCY;
    double l1m_fac = 0;
    if (counts && !mean) l1m_fac = log1p(-lr_fac * (p2stat[0] / p2stat[1] + reg_fac));
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * kBlock) {
        const int i = (int)(x / ld), c = (int)(x - (int64_t)i * ld);
        // l = log(1 - eta); -inf selects the count-weighted mean (rule MF_MERGE_MEAN)
        const double l = !counts ? 0.0
                         : (mean ? -INFINITY
                                 : (c == bias_col ? l1m_bias : (c < n_fac ? l1m_fac : 0.0)));
        const T s0 = snap[x];
        T acc = T(0);
        const double N = counts && !rec ? (double)totals[i] : 0.0;
        const double gN = l != 0.0 && !rec ? -expm1(N * l) : 0.0;
        for (int r = 0; r < n_rep; ++r) {
            const T d = tab[r * stride + x] - s0;
            double w = 1.0;
            if (rec) {  // this rank's steps decayed by the later ranks' steps: (1 - eta)^{N_>r}
                w = exp((double)counts[(int64_t)r * n_items + i] * l);
            } else if (l != 0.0) {
                const double n = (double)counts[(int64_t)r * n_items + i];
                w = n > 0 ? (mean ? n / N : (n / N) * gN / -expm1(n * l)) : 0.0;
            }
            acc += (T)w * d;
        }
        if (apply) {
            const T nv = s0 + acc;
            snap[x] = nv;
            for (int r = 0; r < n_rep; ++r) tab[r * stride + x] = nv;
        }
        if (delta) delta[x] = acc;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void item_apply_kernel(T *tab, T *snap, int64_t total,
                                                            int n_rep, const T *__restrict__ delta)
{
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * kBlock) {
        const T nv = snap[x] + delta[x];
        snap[x] = nv;
        for (int r = 0; r < n_rep; ++r) tab[r * total + x] = nv;
    }
}

// SVD++ y_j across ranks (dist.py): rank r's chunk result is y_r = A_r y_s + c_r (its users'
// end-of-user affine maps composed in CSR order).  phase 0: delta = S_r (y_r - A_r y_s) -- the
// rank's c_r carried through the later ranks' maps; the caller SUM-all-reduces it.  phase 1:
// y = A y_s + delta (A = prod_r A_r) into the table and its snapshot.  a / s: per item, dtype.
template <typename T>
__global__ __launch_bounds__(kBlock) void item_affine_kernel(T *tab, T *snap, int n_items, int ld,
                                                             const T *__restrict__ a,
                                                             const T *__restrict__ s,
                                                             T *__restrict__ delta, int phase)
{
    const int64_t total = (int64_t)n_items * ld;
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * kBlock) {
        const int i = (int)(x / ld);
        if (phase == 0) {
            delta[x] = s[i] * (tab[x] - a[i] * snap[x]);
        } else {
            const T nv = a[i] * snap[x] + delta[x];
            snap[x] = nv;
            tab[x] = nv;
        }
    }
}

// ---------------------------------------------------------------- delta-log merge (MF_MODE_LOG)
//
// After an epoch-chunk in kLog mode, log row k holds the item-row delta d_k of rating k.  The
// merge is a segmented sum in item order: perm lists the chunk's log rows grouped by item (rows
// of an item in increasing k, i.e. the reference's user order), cut into pieces of <= 64 rows
// so the most popular item does not serialise one wave.  Fixed order throughout: the result is
// bit-reproducible.  Then per item, with N = ratings of the item in the chunk (all ranks):
//     q_i += w(N) * sum_k d_k,   w(N) = (1 - (1-eta)^N) / (N eta),
// the count-aware weight for N single steps (every user is its own group): 1 for rare items,
// 1/(N eta) for items whose row would have converged within the chunk (plain SUM
// diverges on ML-1M).  eta as in mf_item_merge.

// The recency-weighted fold (MF_MERGE_RECENCY): the reference applies an item's N steps of a
// chunk one after the other, each on the row the previous ones left.  To first order (the step
// d_k = lr (err_k p_k - reg q) taken at the chunk-start row, the row's own decay eta = lr (<p^2>
// + reg) per step, as in the count-aware weight) the sequential result is
//     q_N - q_0 = sum_k (1 - eta)^(N - 1 - k) d_k       (k = the step's position, users in order)
// -- later steps count more, exactly as they do in the reference; the count-aware weight is this
// with every step given the mean weight.  The replay / reduce weight each rating's gradient by
// its (1 - eta)^(N - 1 - pos) (eta of the bias column for the bias, of the factor columns else),
// and mf_log_apply adds lr (S - reg q sum_k (1 - eta)^(N-1-k)).
struct Recency {
    const int32_t *rpos;    // per log entry (parallel to perm): position among this rank's
                            // ratings of the chunk of the same item, users in order; NULL: off
    const int32_t *pos0;    // per item: the chunk's ratings of the item on earlier ranks (NULL: 0)
    const int32_t *totals;  // per item: N, the chunk's ratings of the item on every rank
    const double *p2stat;   // {sum p^2, count} at the chunk start (every rank)
    double lr_qi, reg_qi, eta_b;
};

// log(1 - eta) of the factor columns and of the bias column
__device__ __forceinline__ void recency_logs(const Recency &rc, double &l_q, double &l_b)
{
    const double n = rc.p2stat[1];
    const double p2 = n > 0 ? rc.p2stat[0] / n : 0.0;
    l_q = log1p(-rc.lr_qi * (p2 + rc.reg_qi));
    l_b = log1p(-rc.eta_b);
}

// this lane's entry x of a piece of `item`: (1 - eta)^(N - 1 - pos) for both column kinds
template <typename T>
__device__ __forceinline__ void recency_weights(const Recency &rc, double l_q, double l_b,
                                                int item, int x, T &wf, T &wb)
{
    const double back = (double)(rc.totals[item] - 1 - rc.rpos[x] - (rc.pos0 ? rc.pos0[item] : 0));
    wf = (T)exp(back * l_q);
    wb = (T)exp(back * l_b);
}

// per lane and lane group: 1 in the element that holds column c_bias, else 0
template <typename T, int G>
__device__ __forceinline__ void bias_selector(int c_bias, typename Lane8<T>::vec (&bsel)[G])
{
    using L = Lane8<T>;
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int v = 0; v < G; ++v)
#pragma unroll
        for (int e = 0; e < L::W; ++e)
            L::set(bsel[v], e, (lane + kWave * v) * L::W + e == c_bias ? T(1) : T(0));
}

// One wave per TWO pieces (<= 64 rows each) at a time: each piece's log-row indices arrive with
// ONE vector load (lane l holds perm[beg + l]) and are broadcast with v_readlane, so the row
// gathers carry no scalar-load round trips; rows are read 8 per piece at a time (16 in flight) in
// the 8-byte lane layout of the epoch kernel (one dwordx2 per lane per 512 B of row).  Two pieces
// per iteration: most pieces are short (the C5 shard's chunks hold ~8 ratings per item), so a
// piece costs its chain of dependent loads (bounds -> rows, item -> N), which the second piece's
// overlap.  REC: each row weighted by its recency weight.
template <typename T, int G, bool REC>
__global__ __launch_bounds__(kBlock) void log_reduce_kernel(
    const T *__restrict__ qlog, int ld, int n_cols, const int32_t *__restrict__ perm,
    const int32_t *__restrict__ piece_beg, int64_t n_pieces, T *__restrict__ sums,
    const int32_t *__restrict__ items, const int32_t *__restrict__ piece_item, Recency rc,
    int bias_col)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    double l_q = 0, l_b = 0;
    vec bsel[G];
    if constexpr (REC) {
        recency_logs(rc, l_q, l_b);
        bias_selector<T, G>(bias_col, bsel);
    }
    constexpr int kP = 2;   // pieces per iteration
    constexpr int kU = 8;   // rows in flight per piece
    for (int64_t pc0 = wave; pc0 < n_pieces; pc0 += kP * n_waves) {
        int cnt[kP], myk[kP];
        T wf_l[kP], wb_l[kP];
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            const int64_t pc = pc0 + q * n_waves;
            const bool ok = pc < n_pieces;  // (uniform)
            const int64_t pcc = ok ? pc : pc0;
            const int beg = piece_beg[pcc];
            cnt[q] = ok ? piece_beg[pcc + 1] - beg : 0;  // 1 <= cnt <= 64 for a real piece
            const int c1 = cnt[q] > 0 ? cnt[q] : 1;
            const int xr = beg + (lane < c1 ? lane : c1 - 1);
            myk[q] = perm[xr];
            wf_l[q] = T(1);
            wb_l[q] = T(1);
            if constexpr (REC) {
                const int item = piece_item ? piece_item[pcc] : items[readlane(myk[q], 0)];
                recency_weights(rc, l_q, l_b, item, xr, wf_l[q], wb_l[q]);
            }
        }
        vec acc[kP][G];
#pragma unroll
        for (int q = 0; q < kP; ++q)
#pragma unroll
            for (int v = 0; v < G; ++v) acc[q][v] = L::splat(T(0));
        const int cmax = cnt[0] > cnt[1] ? cnt[0] : cnt[1];
        for (int x = 0; x < cmax; x += kU) {
            vec g[kP][kU][G];
#pragma unroll
            for (int q = 0; q < kP; ++q) {
                const int cq = cnt[q] > 0 ? cnt[q] : 1;
#pragma unroll
                for (int a = 0; a < kU; ++a) {
                    const int k = readlane(myk[q], x + a < cq ? x + a : cq - 1);
                    const T *row = qlog + (int64_t)k * ld;
#pragma unroll
                    for (int v = 0; v < G; ++v) {  // (lanes past the row re-read column 0)
                        const int c0 = (lane + kWave * v) * W;
                        g[q][a][v] = *(const vec *)(row + (c0 < ld ? c0 : 0));
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < kP; ++q)
#pragma unroll
                for (int a = 0; a < kU; ++a)
                    if (x + a < cnt[q]) {
                        if constexpr (REC) {
                            const int xa = x + a < kWave ? x + a : kWave - 1;
                            const T wf = readlane(wf_l[q], xa), wb = readlane(wb_l[q], xa);
#pragma unroll
                            for (int v = 0; v < G; ++v)
                                acc[q][v] += (L::splat(wf) + (wb - wf) * bsel[v]) * g[q][a][v];
                        } else {
#pragma unroll
                            for (int v = 0; v < G; ++v) acc[q][v] += g[q][a][v];
                        }
                    }
        }
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            if (cnt[q] <= 0) continue;
            const int64_t pc = pc0 + q * n_waves;
#pragma unroll
            for (int v = 0; v < G; ++v) {
                const int c0 = (lane + kWave * v) * W;
#pragma unroll
                for (int e = 0; e < W; ++e)
                    if (c0 + e < ld) sums[pc * ld + c0 + e] = c0 + e < n_cols ? L::get(acc[q][v], e) : T(0);
            }
        }
    }
}

#ifndef MF_EPOCH_WPC
#define MF_EPOCH_WPC 64  // epoch kernel: default cap on waves per CU
#endif
#ifndef MF_REPLAY_U
#define MF_REPLAY_U 16  // ratings per replay group (two groups in flight)
#endif
#ifndef MF_REPLAY_WPC
#define MF_REPLAY_WPC 16  // replay waves per CU
#endif
#ifndef MF_REPLAY_ROW_NT
// the replay's checkpoint-row gathers non-temporal: each row is read twice, far apart, so caching
// it buys nothing, and streaming it past the MALL leaves the error log's lines there for the
// error gathers (C4 replay fp32 12.8 -> 12.1 ms, fp64 18.9 -> 17.9; profiles/r5n_replay_nt.txt)
#define MF_REPLAY_ROW_NT 1
#endif

// ---------------------------------------------------------------- the per-item fold
//
// One item of mf_log_apply: its piece sums in a fixed order -- sums' pieces [a0, a1), then (TWO)
// sums2's [b0, b1) -- then q += lr (S - W reg q) by the merge rule.  Run by log_apply_kernel (one
// wave per item) and by the replay wave that completes an item's last piece (mf_launch_fold);
// COH: the piece sums read at the agent's coherence point (written by waves of launches still
// running).  KU pieces in flight per group; the sum order does not depend on it.
struct FoldRule {
    int count_rule;
    double eta_fac, l_fac, l_bias, eta_bias, lr_f, reg_f, lr_b, reg_b;
};
__device__ __forceinline__ FoldRule fold_rule(int count_rule, const double *p2stat, double eta_bias,
                                              double lr_fac, double reg_fac, double lr_f,
                                              double reg_f, double lr_b, double reg_b)
{
    FoldRule r{count_rule, 0, 0, 0, eta_bias, lr_f, reg_f, lr_b, reg_b};
    if (count_rule) {
        r.eta_fac = lr_fac * (p2stat[0] / p2stat[1] + reg_fac);
        r.l_fac = log1p(-r.eta_fac);
        r.l_bias = log1p(-eta_bias);
    }
    return r;
}
template <typename T, bool COH>
__device__ __forceinline__ T fold_ld(const T *p)
{
    if constexpr (COH)
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        return *p;
}
template <typename T, int V, bool TWO, bool COH, int KU>
__device__ __forceinline__ void apply_item(
    int64_t i, int lane, T *__restrict__ qb, int ld, int n_fac, int bias_col,
    const T *__restrict__ sums, const int32_t *__restrict__ item_piece_ptr,
    const T *__restrict__ sums2, const int32_t *__restrict__ item_piece_ptr2,
    const int32_t *__restrict__ totals, const FoldRule &r, T *__restrict__ delta_out, int apply,
    T *__restrict__ bias_out)
{
    // every load that does not depend on another first: both groups' piece ranges, the count and
    // the item row; then the first KU pieces of each group together
    const int a0 = item_piece_ptr ? item_piece_ptr[i] : (int)i;
    const int a1 = item_piece_ptr ? item_piece_ptr[i + 1] : (int)i + 1;
    const int b0 = TWO ? item_piece_ptr2[i] : 0, b1 = TWO ? item_piece_ptr2[i + 1] : 0;
    const double N = totals ? (double)totals[i] : 0.0;
    T q[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + kWave * v;
        q[v] = apply && c < ld ? qb[i * ld + c] : T(0);
    }
    auto load = [&](const T *__restrict__ sp, int pc, int p1, T (&g)[KU][V]) {
#pragma unroll
        for (int a = 0; a < KU; ++a)
#pragma unroll
            for (int v = 0; v < V; ++v)
                g[a][v] = (pc + a < p1 && lane + kWave * v < ld)
                              ? fold_ld<T, COH>(sp + (int64_t)(pc + a) * ld + lane + kWave * v)
                              : T(0);
    };
    T acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = T(0);
    auto add = [&](T (&g)[KU][V]) {
#pragma unroll
        for (int a = 0; a < KU; ++a)
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] += g[a][v];
    };
    // the item's pieces in sums, then (split log) its pieces in sums2, in that fixed order
    T ga[KU][V];
    load(sums, a0, a1, ga);
    if constexpr (TWO) {
        T gb[KU][V];
        load(sums2, b0, b1, gb);
        add(ga);
        for (int pc = a0 + KU; pc < a1; pc += KU) {
            load(sums, pc, a1, ga);
            add(ga);
        }
        add(gb);
        for (int pc = b0 + KU; pc < b1; pc += KU) {
            load(sums2, pc, b1, gb);
            add(gb);
        }
    } else {
        add(ga);
        for (int pc = a0 + KU; pc < a1; pc += KU) {
            load(sums, pc, a1, ga);
            add(ga);
        }
    }
    // the count-aware weights (one per column kind, the same for every factor column);
    // recency (count_rule 2): the sums arrive weighted, the reg term takes the weights' sum
    // sum_k (1 - eta)^(N-1-k) = (1 - (1 - eta)^N) / eta = w N
    double w_fac = 1.0, w_bias = 1.0;
    if (r.count_rule && N > 1.0) {
        w_fac = -expm1(N * r.l_fac) / (N * r.eta_fac);
        w_bias = -expm1(N * r.l_bias) / (N * r.eta_bias);
    }
    const bool rec = r.count_rule == 2;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = lane + kWave * v;
        if (c >= ld) continue;
        const int64_t x = i * ld + c;
        if (delta_out) delta_out[x] = acc[v];
        if (apply && (c < n_fac || c == bias_col)) {
            const bool b = c == bias_col;
            const double w = b ? w_bias : w_fac;
            // the log holds gradients g_k = err_k pe_k: sum_k d_k = lr (S - N reg q)
            T nq;
            if (rec) {
                nq = q[v] + (T)(b ? r.lr_b : r.lr_f) *
                                (acc[v] - (T)(w * N) * (T)(b ? r.reg_b : r.reg_f) * q[v]);
            } else {
                const T d = (T)(b ? r.lr_b : r.lr_f) *
                            (acc[v] - (T)N * (T)(b ? r.reg_b : r.reg_f) * q[v]);
                nq = q[v] + (T)w * d;
            }
            qb[x] = nq;
            if (b && bias_out) bias_out[i] = nq;  // (the item-bias mirror of the SB epoch)
        }
    }
}

// ---------------------------------------------------------------- checkpoint-log replay
//
// The SVD log in checkpoint form (mf_svd_epoch with elog != NULL): per pair (c, c + 1) of a
// user's ratings (c - row_ptr[u] even) log row c holds p_{c+1}, the user row AFTER rating c
// (for a user's odd last rating c: the final row), and elog[k] = err_k for every rating.  The
// gradient of rating k is g_k = err_k p_k (p_k = the row before rating k):
//   k = c + 1:  p_k = row c, as stored;
//   k = c:      p_k = (p_{c+1} - err_c lrp o q_{i_c}) / ap  -- the epoch kernel's step
//               p_{c+1} = ap o p_c + err_c lrp o q_{i_c} undone (ap = 1 - lr_pu reg_pu on factor
//               columns, 1 elsewhere; lrp = lr_pu on factor columns, 0 elsewhere).
// A piece holds ratings of ONE item, so q_{i_c} is the piece's own (snapshot) item row: one
// load per piece, and the replay gathers nothing but the checkpoint rows (no item rows, no item
// ids).  Summed per piece in perm order exactly like log_reduce_kernel; equal to the gradient
// log's sums up to a rounding of the undone step (fp64: the delta-log oracle to 1e-9).
// One wave per piece (any number of ratings of one item, 64 at a time: lane x holds rating x's
// checkpoint offset, parity, err and weight, vector gathers once per 64).  Pieces longer than 64
// shorten mf_log_apply's per-item chain of piece rows (C4's top item: ~1M ratings = 16k pieces
// of 64).  Odd and even ratings are summed apart, so a
// rating costs two v_readlane broadcasts, the row gather and 2 (packed) FMAs per element; the
// undone step enters once per piece: sum_even w err_k p_k = iap o (sum_even w err p_{c+1} -
// D sum_even w err^2).  Two groups of MF_REPLAY_U rows are in flight per wave.
template <typename T, int G, bool REC, bool FOLD = false>
__device__ __forceinline__ void log_replay_body(
    const T *__restrict__ ckpt, const T *__restrict__ elog, int ldq, int K,
    const int32_t *__restrict__ items, const T *__restrict__ qb, int n_items, T lr_pu, T inv_ap,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ ck_pos,
    const int32_t *__restrict__ piece_beg, int64_t n_pieces, T *__restrict__ sums, int err_col,
    const int32_t *__restrict__ piece_item, const int64_t wave, const int64_t n_waves,
    const bool wt, const Recency &rc, const int ldc, const mf_ext::FoldArgs &fa)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    constexpr int kU = MF_REPLAY_U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t qrow = (uint32_t)ldq * sizeof(T), q_oob = (uint32_t)n_items * qrow;
    const rsrc_t q_rs = make_rsrc(qb, q_oob);
    uint32_t cq[G];
    int cc[G];
    vec lrp[G], iap[G];
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;
        cq[v] = c0 < ldq ? (uint32_t)c0 * sizeof(T) : q_oob;
        cc[v] = c0 < ldc ? c0 : 0;  // (lanes past the row re-read column 0: no branch)
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const bool fac = c0 + e < K;
            L::set(lrp[v], e, fac ? lr_pu : T(0));
            L::set(iap[v], e, fac ? inv_ap : T(1));
        }
    }
    double l_q = 0, l_b = 0;
    vec bsel[G];
    bias_selector<T, G>(K, bsel);
    if constexpr (REC) recency_logs(rc, l_q, l_b);
    // narrow rows (MF_EPOCH_CKPT_NARROW): the K factor columns only; the bias column's gradient
    // err_k * 1 is summed from the per-lane errors
    const bool narrow = ldc < ldq;
    // lane groups the checkpoint rows fill (G = kLaMaxG + 1 only with narrow rows of kLaMaxG
    // groups -- fp64 K = 128 -- whose last group holds the bias column alone)
    constexpr int GR = G > kLaMaxG ? kLaMaxG : G;
    // the fold inside the replay (mf_launch_fold): the wave that completes an item's last piece
    // -- of either launch group -- applies the item (apply_item, mf_log_apply's arithmetic)
    constexpr bool fold = FOLD;
    FoldRule fr{};
    if constexpr (fold)
        fr = fold_rule(fa.count_rule, fa.p2stat, fa.eta_b, fa.lr_c, fa.reg_c, fa.lr_f, fa.reg_f,
                       fa.lr_b, fa.reg_b);
    for (int64_t pc = wave; pc < n_pieces; pc += n_waves) {
        // a piece: >= 1 ratings of ONE item, taken 64 at a time (lane x: rating x of the
        // sub-piece); the undone step's and the bias column's scalar sums accumulate per lane
        const int pbeg = piece_beg[pc], pend = piece_beg[pc + 1];
        // the piece's item row (snapshot) -> D = lrp o q_i
        // (piece_item: the item id without the perm -> items hop on the piece's critical path)
        const int item = piece_item ? piece_item[pc] : items[perm[pbeg]];
        const uint32_t qoff = (uint32_t)item * qrow;
        vec D[G];
#pragma unroll
        for (int v = 0; v < G; ++v) D[v] = lrp[v] * L::template lds<0>(q_rs, cq[v], qoff);
        vec ao[G], ae[G];
#pragma unroll
        for (int v = 0; v < G; ++v) ao[v] = ae[v] = L::splat(T(0));
        T se_l = T(0), sb_l = T(0);  // per lane: sum_even w err^2, the bias column's extra
        for (int beg = pbeg; beg < pend; beg += kWave) {
            const int cnt = pend - beg < kWave ? pend - beg : kWave;  // 1 <= cnt <= 64
            const int xl = beg + (lane < cnt ? lane : cnt - 1);
            // lane x: rating x, its pair's (packed) checkpoint row and parity (2 row + odd)
            const int k_l = perm[xl], ck_l = ck_pos[xl];
            const int c_l = ck_l >> 1, odd_l = ck_l & 1;  // odd 1: k = c + 1 (the row as stored)
            // err_k per lane: from elog, or (err_col > 0) column err_col + odd of its checkpoint
            // row (one gather per lane: the line is the row load's own); lanes >= cnt: 0
            const T ek_l = lane >= cnt ? T(0)
                           : err_col > 0 ? ckpt[(int64_t)c_l * ldc + err_col + odd_l] : elog[k_l];
            // gradient weight per lane: err_k, times (REC) its recency weight wf for the factor
            // columns; the bias column (p_k's column K is 1, so its gradient is err_k) gets
            // sum err_k (wb - wf) added once per piece.
            T ef_l = ek_l;
            if constexpr (REC) {
                T wf_l, wb_l;
                recency_weights(rc, l_q, l_b, item, xl, wf_l, wb_l);
                ef_l = ek_l * wf_l;
                sb_l += ek_l * (wb_l - wf_l);
            }
            if (narrow) sb_l += ef_l;  // (the bias column read nothing: all of it here)
            // g_k = p_k for odd k, iap o (p_{c+1} - err_k D) for even: split by parity so a
            // rating costs one FMA per element --
            // acc = sum_odd ef p + iap o (sum_even ef p - D sum_even ef ek)
            const T eo_l = odd_l ? ef_l : T(0), ee_l = odd_l ? T(0) : ef_l;
            se_l += ee_l * ek_l;
            auto load_grp = [&](const int x0, vec (&p)[kU][G]) {
#pragma unroll
                for (int y = 0; y < kU; ++y) {  // (x past cnt: lane cnt-1's rating, weight 0)
                    const int x = x0 + y < kWave ? x0 + y : kWave - 1;
                    const T *row = ckpt + (int64_t)readlane(c_l, x) * ldc;
#pragma unroll
                    for (int v = 0; v < GR; ++v)
#if MF_REPLAY_ROW_NT
                        p[y][v] = __builtin_nontemporal_load((const vec *)(row + cc[v]));
#else
                        p[y][v] = *(const vec *)(row + cc[v]);
#endif
                }
            };
            auto comp_grp = [&](const int x0, vec (&p)[kU][G]) {
#pragma unroll
                for (int y = 0; y < kU; ++y) {
                    const int x = x0 + y < kWave ? x0 + y : kWave - 1;
                    const T wo = readlane(eo_l, x), we = readlane(ee_l, x);
#pragma unroll
                    for (int v = 0; v < GR; ++v) {
                        ao[v] += wo * p[y][v];
                        ae[v] += we * p[y][v];
                    }
                }
            };
            vec pA[kU][G], pB[kU][G];
            load_grp(0, pA);
            for (int x0 = 0; x0 < cnt; x0 += 2 * kU) {
                load_grp(x0 + kU, pB);
                comp_grp(x0, pA);
                if (x0 + kU >= cnt) break;
                load_grp(x0 + 2 * kU, pA);
                comp_grp(x0 + kU, pB);
            }
        }
        const T se = wave_sum_u(se_l);
        const T sb = REC || narrow ? wave_sum_u(sb_l) : T(0);
        vec acc[G];
#pragma unroll
        for (int v = 0; v < G; ++v) {
            acc[v] = ao[v] + iap[v] * (ae[v] - se * D[v]);
            if (narrow) acc[v] -= acc[v] * bsel[v];
            acc[v] += sb * bsel[v];
        }
#pragma unroll
        for (int v = 0; v < G; ++v) {
            const int c0 = (lane + kWave * v) * W;
#pragma unroll
            for (int e = 0; e < W; ++e)
                if (c0 + e < ldq) {
                    const T x = c0 + e <= K ? L::get(acc[v], e) : T(0);
                    if (wt)  // (written through to the agent's coherence point: mf_launch_join)
                        __hip_atomic_store(&sums[pc * ldq + c0 + e], x, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    else
                        sums[pc * ldq + c0 + e] = x;
                }
        }
        if constexpr (fold) {
            // this piece's sums have reached the coherence point before the item's count moves;
            // the wave that moves it to the item's piece total is the last and folds the item
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int last = 0;
            if (lane == 0) {
                const int n = (fa.ipp_a[item + 1] - fa.ipp_a[item]) +
                              (fa.ipp_b ? fa.ipp_b[item + 1] - fa.ipp_b[item] : 0);
                const int old = __hip_atomic_fetch_add(fa.cnt + item, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                if (old == n - 1) {
                    __hip_atomic_store(fa.cnt + item, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last = 1;
                }
            }
            if (__builtin_amdgcn_readfirstlane(last)) {
                constexpr int VA = G * W;  // (>= mf_log_apply's ceil(ld / 64): masked past ld)
                if (fa.ipp_b)
                    apply_item<T, VA, true, true, 4>(
                        item, lane, (T *)fa.qb, fa.ld, fa.n_fac, fa.bias_col, (const T *)fa.sums_a,
                        fa.ipp_a, (const T *)fa.sums_b, fa.ipp_b, fa.totals, fr, nullptr, 1,
                        (T *)fa.bias_out);
                else
                    apply_item<T, VA, false, true, 4>(
                        item, lane, (T *)fa.qb, fa.ld, fa.n_fac, fa.bias_col, (const T *)fa.sums_a,
                        fa.ipp_a, nullptr, nullptr, fa.totals, fr, nullptr, 1, (T *)fa.bias_out);
            }
        }
    }
}


// In-kernel join of the two-stream SVD step (mf_launch_join): the light replay (role 1) and the
// heavy replay (role 2) of one chunk meet without a barrier packet in the main stream's queue.
// Per-launch arrival counters of roles 1 / 2 (reset by their last arrivals), the epoch id of the
// last light replay that completed and a timed-out-wait flag (layout below).  Role 1: every block arrives after its stores (release); the last one publishes the epoch.
// Role 2: the last block to arrive waits (one lane, bounded) until the light replay of the same
// epoch has published, so the kernel queued after the heavy replay (the fold) sees both groups'
// sums.  Only the LAST block of role 2 waits: every other block has exited, so a light replay
// that has not started yet still finds room to run.  Role 1's sums are stored as agent-scope
// atomic stores (written through each XCD's L2) and every block waits for its stores before it
// arrives with a RELAXED add: a release fence per block (an L2 write-back each) made the light
// replay 72 -> 125 us; the only fences are the publishing store's and the waiter's acquire.
constexpr int kJoinSpinMax = 1 << 22;  // (~0.4 s of s_sleep: a wait that never ends is an error)
// word layout (uint32, each counter on its own 128-byte line): role r's arrival counters for the
// eight residue classes of blockIdx (mod 8) at kJoinSub<r> + 32 c, its top counter at kJoinTop<r>;
// the published epoch at kJoinFlag, the timeout flag at kJoinErr.  Two levels: ~G/8 same-address
// atomics per class in parallel, then <= 8 at the top (one counter for ~1000 blocks serialised
// the blocks' arrivals behind each other at the end of the launch).
constexpr int kJoinSub1 = 0, kJoinTop1 = 256, kJoinSub2 = 288, kJoinTop2 = 544;
constexpr int kJoinFlag = 576, kJoinErr = 608;
__device__ __forceinline__ bool join_count(uint32_t *w, uint32_t n) {  // true: the n-th arrival
    const uint32_t old = __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old != n - 1) return false;
    __hip_atomic_store(w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}
__device__ __forceinline__ void join_arrive(uint32_t *join, int role, uint32_t epoch)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's stores have completed)
    __syncthreads();  // (... and every wave's, before the block arrives)
    if (threadIdx.x != 0) return;
    const uint32_t G = gridDim.x, c = blockIdx.x & 7;
    if (!join_count(join + (role == 1 ? kJoinSub1 : kJoinSub2) + 32 * c, (G - c + 7) / 8)) return;
    if (!join_count(join + (role == 1 ? kJoinTop1 : kJoinTop2), G < 8 ? G : 8)) return;
    if (role == 1) {
        __hip_atomic_store(join + kJoinFlag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (int spins = 0;; ++spins) {
        const uint32_t done = __hip_atomic_load(join + kJoinFlag, __ATOMIC_ACQUIRE,
                                                __HIP_MEMORY_SCOPE_AGENT);
        if ((int32_t)(done - epoch) >= 0) break;
        if (spins >= kJoinSpinMax) {
            __hip_atomic_store(join + kJoinErr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// The in-replay fold's last step: the next chunk's <p^2> statistic, summed by the last block to
// finish of the fold's launches (two levels of arrival counters per launch, as join_arrive, then
// one over the launches); no block waits.  Both epoch kernels have ended by then (each launch
// follows its own group's epoch), so user_sq is final; it is read at the coherence point.
__device__ __forceinline__ void fold_arrive(const mf_ext::FoldArgs &fa)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        int last = 0;
        const uint32_t G = gridDim.x, c = blockIdx.x & 7;
        uint32_t *w = fa.blk + 320 * (fa.role - 1);
        if (join_count(w + 32 * c, (G - c + 7) / 8) && join_count(w + 256, G < 8 ? G : 8))
            last = join_count(fa.blk + 640, (uint32_t)fa.n_launch) ? 1 : 0;
        s_last = last;
    }
    __syncthreads();
    if (s_last) block_sum_sq<true>(fa.user_sq, fa.n_users, fa.n_fac, fa.stat_next);
}

template <typename T, int G, bool REC, bool FOLD>
__global__ __launch_bounds__(kBlock) void log_replay_kernel(
    const T *__restrict__ ckpt, const T *__restrict__ elog, int ldq, int K,
    const int32_t *__restrict__ items, const T *__restrict__ qb, int n_items, T lr_pu, T inv_ap,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ ck_pos,
    const int32_t *__restrict__ piece_beg, int64_t n_pieces, T *__restrict__ sums, int xmask,
    int err_col, const int32_t *__restrict__ piece_item, uint32_t *join, int join_role,
    uint32_t join_epoch, Recency rc, int ldc, mf_ext::FoldArgs fa)
{
    int64_t wave, n_waves;
    if (wave_slot(xmask, wave, n_waves)) {
        SlotSettle settle((threadIdx.x & (kWave - 1)) == 0 ? xmask : 0, wave, n_waves,
                          wave_grid_index());
        log_replay_body<T, G, REC, FOLD>(ckpt, elog, ldq, K, items, qb, n_items, lr_pu, inv_ap,
                                         perm, ck_pos, piece_beg, n_pieces, sums, err_col,
                                         piece_item, wave, n_waves,
                                         FOLD || (join && join_role == 1), rc, ldc, fa);
    }
    if (join) join_arrive(join, join_role, join_epoch);
    if constexpr (FOLD) {
        if (fa.stat_next) fold_arrive(fa);
    }
}

#ifndef MF_APPLY_U
#define MF_APPLY_U 16  // mf_log_apply: piece rows in flight per wave (a popular item has ~60)
#endif
template <typename T, int V, bool TWO>  // TWO: a split chunk (sums2, the heavy group's pieces)
__global__ __launch_bounds__(kBlock) void log_apply_kernel(
    T *__restrict__ qb, int n_items, int ld, int n_fac, int bias_col, const T *__restrict__ sums,
    const int32_t *__restrict__ item_piece_ptr, const T *__restrict__ sums2,
    const int32_t *__restrict__ item_piece_ptr2, const int32_t *__restrict__ totals,
    int count_rule, double eta_bias, double lr_fac, double reg_fac, double lr_f, double reg_f,
    double lr_b, double reg_b, const double *__restrict__ p2stat, T *__restrict__ delta_out,
    int apply, double *__restrict__ stat_next, const double *__restrict__ user_sq, int64_t n_sq,
    int sq_cols, T *__restrict__ bias_out)
{
    // the next chunk's {sum |p_u|^2, count}: the launch's extra FIRST block, which does no item
    // (dispatched first: at 2M users the one-block sum is the launch's longest piece of work)
    if (stat_next && blockIdx.x == 0) {
        if (user_sq) {
            block_sum_sq(user_sq, n_sq, sq_cols, stat_next);
        } else if (threadIdx.x < 2) {
            stat_next[threadIdx.x] = 0.0;  // (cleared for the next chunk's mf_sumsq)
        }
        return;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int blk0 = stat_next ? 1 : 0;  // (block 0: the statistic)
    const int64_t wave = (int64_t)(blockIdx.x - blk0) * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)(gridDim.x - blk0) * kBlock) / kWave;
    const FoldRule r = fold_rule(count_rule, p2stat, eta_bias, lr_fac, reg_fac, lr_f, reg_f, lr_b,
                                 reg_b);
    for (int64_t i = wave; i < n_items; i += n_waves)
        apply_item<T, V, TWO, false, MF_APPLY_U>(i, lane, qb, ld, n_fac, bias_col, sums,
                                                 item_piece_ptr, sums2, item_piece_ptr2, totals, r,
                                                 delta_out, apply, bias_out);
}

// ---------------------------------------------------------------- blocked solve (heaviest users)
//
// SVD checkpoint log with the errors in the rows, one WORKGROUP per user.  The lookahead body
// pays ~48 instructions per rating on one wave (two 64-lane reductions): the heaviest user's
// chain of 1805 ratings is the ML-1M step's critical path.  Unrolled over a block of kGB = 16
// ratings that starts at the user row P (column K: the constant 1 of the item bias, K+1:
// c = mu + bu), the reference recursion (mf.pyx:247-262) makes every error a linear function of
// the block's earlier errors:
//   err_m = rhs_m - sum_{t<m} L_mt err_t
//   rhs_m = r_m - a^m <q_m, P>_fac - q_m[K] P[K] - abu^m c - kb (1 + abu + ... + abu^(m-1))
//   L_mt  = a^(m-1-t) lr_pu <q_m, q_t>_fac + abu^(m-1-t) lr_bu
// (a = 1 - lr_pu reg_pu, abu = 1 - lr_bu reg_bu, kb = mu (1 - abu); column K+1 of every item row
// is 1).  Per block: wave 0 solves the 16 errors (16 x readlane + FMA -- no reduction on the
// chain) while waves 1-3 build the NEXT block's Gram matrix <q_m, q_t> with MFMA (16x16x4) and
// gather the block after it into LDS; then every wave runs the row recursion with lane = column
// (the checkpoint rows of the block's pairs, its end row) and the next block's <q_m, P>.  Same
// arithmetic as the lookahead body up to rounding: fp64 equals oracle_svd_sgd_deltalog to 1e-9.
constexpr int kGB = 16;  // ratings per block (one 16x16 MFMA tile)
template <typename T>
struct GramCols { static constexpr int n = 1024 / (int)sizeof(T); };  // rows of <= 1 KiB

template <typename T>
struct GramMfma;
template <>
struct GramMfma<double> {
    typedef double acc __attribute__((ext_vector_type(4)));
    __device__ static __forceinline__ acc step(double a, double b, acc c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 r
    __device__ static __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <>
struct GramMfma<float> {
    typedef float acc __attribute__((ext_vector_type(4)));
    __device__ static __forceinline__ acc step(float a, float b, acc c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // the standard 16x16 C/D map: col = lane & 15, row = 4 (lane >> 4) + r
    __device__ static __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

// a workgroup barrier that orders LDS only: __syncthreads() also waits for every outstanding
// global load and store (vmcnt(0)), which would drain the row prefetches and the checkpoint-row
// stores at every one of the block's three barriers
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

constexpr int kGWin = 1024;  // item ids / ratings of a user staged in LDS at a time
constexpr int kGSlots = 4;   // item-row blocks in the LDS ring: b, b+1, b+2, and b+3 in flight

// LDS bytes of the dynamic ring of mf_svd_gram_kernel (kGSlots blocks of kGB rows)
int gram_ring_bytes(int ldq, int esz) { return kGSlots * kGB * ldq * esz; }

template <typename T>
__global__ __launch_bounds__(kBlock) void mf_svd_gram_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, int ldu, const T *__restrict__ qb, int ldq, int K,
    int biased, Hyper<T> hp, T *__restrict__ qlog, double *__restrict__ psq, int err_col,
    int xmask)
{
    // the block ring: kGSlots x kGB item rows packed at stride ldq (LDS-DMA writes 1-KiB pieces
    // lane-linearly, and a block of 16 rows of a 64-byte multiple is whole pieces)
    extern __shared__ __attribute__((aligned(16))) char gram_ring[];
    __shared__ T gp[3][kGB][kGB];     // the helpers' partial Gram matrices
    __shared__ T lm[2][kGB][kGB];     // L of the current / next block
    __shared__ T pw[3][kGB + 1];      // a^k, abu^k, kb (1 + .. + abu^(k-1))
    __shared__ T E[kGB], X0[kGB], P[GramCols<T>::n];
    __shared__ int32_t ids[kGWin];    // item ids / ratings [win0, win0 + kGWin) of the user
    __shared__ T rtw[kGWin];
    __shared__ double sqw[kBlock / kWave];
    using MF = GramMfma<T>;
    const int tid = threadIdx.x, w = tid / kWave, lane = tid & (kWave - 1);
    const int wu = __builtin_amdgcn_readfirstlane(w);
    int64_t slot = blockIdx.x, n_slots = gridDim.x;
    if (xmask) {  // this block's slot among the launch's blocks on the XCDs of xmask
        const int x = __builtin_amdgcn_readfirstlane(xcc_id());
        const bool in = (xmask >> x) & 1;
        const int c = __builtin_popcount(xmask), rank = __builtin_popcount(xmask & ((1 << x) - 1));
        slot = in ? (int64_t)(blockIdx.x >> 3) * c + rank : -1;
        n_slots = (int64_t)(gridDim.x >> 3) * c;
        if (!in) {
            if (tid == 0) dispatch_settle(blockIdx.x, -1, n_slots);  // (the dispatch check)
            return;
        }
    }
    // (the block's settlement, by thread 0 when the block ends)
    SlotSettle settle(tid == 0 ? xmask : 0, slot, n_slots, blockIdx.x);
    const T lr_bu = biased ? hp.lr_bu : T(0);
    const T a = T(1) - hp.lr_pu * hp.reg_pu, abu = T(1) - lr_bu * hp.reg_bu;
    const T kb = hp.gm * (T(1) - abu);
    if (tid <= kGB) {
        T x = T(1), y = T(1), g = T(0);
        for (int t = 0; t < tid; ++t) {
            g += kb * y;
            x *= a;
            y *= abu;
        }
        pw[0][tid] = x;
        pw[1][tid] = y;
        pw[2][tid] = g;
    }
    // the row recursion's column (waves 0, 2, 3: wave 1 issues the LDS-DMA and keeps its memory
    // counter to those loads) and its constants (ap, lrp, kvec of epoch_body_la)
    const int c = w == 0 ? lane : (w >= 2 ? (w - 1) * kWave + lane : -1);
    const bool col = c >= 0 && c < ldq;
    const bool fac = c >= 0 && c < K, ub = c == K + 1;
    const T apc = fac ? a : (ub ? abu : T(1));
    const T lrpc = fac ? hp.lr_pu : (ub ? lr_bu : T(0));
    const T kvc = ub ? kb : T(0);
    const int nk = (K + 3) / 4;  // MFMA k-steps over the factor columns
    const uint32_t rowb = (uint32_t)ldq * sizeof(T);
    const int pieces = (int)(kGB * rowb / 1024);  // LDS-DMA instructions per block
    auto ring = [&](int b) -> T * { return (T *)(gram_ring + (size_t)(b % kGSlots) * kGB * rowb); };

    for (int64_t sidx = slot; sidx < n_sched; sidx += n_slots) {
        const int u = sched[sidx];
        if (u < 0) continue;
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        if (n <= 0) continue;
        const int nb = (n + kGB - 1) / kGB;
        const int32_t *__restrict__ it = items + s;
        const T *__restrict__ rr = ratings + s;
        T *__restrict__ lrows = qlog + ck_row0(s, u) * ldq;
        int win0 = 0;
        auto load_win = [&](int j0) {  // every thread: the id / rating window from rating j0
            win0 = j0;
            for (int x = tid; x < kGWin && j0 + x < n; x += kBlock) {
                ids[x] = it[j0 + x];
                rtw[x] = rr[j0 + x];
            }
        };
        // wave 1: block b's rows gathered by index into its ring slot (global_load_lds, 16 B
        // per lane: piece i of the block is bytes [1024 i, 1024 (i + 1)) of its packed rows)
        auto dma = [&](int b) {
            const char *q8 = (const char *)qb;
            char *dst = (char *)ring(b);
            for (int i = 0; i < pieces; ++i) {
                const uint32_t x = (uint32_t)i * 1024u + (uint32_t)lane * 16u;
                const int r = (int)(x / rowb);
                const uint32_t cb = x - (uint32_t)r * rowb;
                const int j = b * kGB + r;
                const int64_t id = ids[(j < n ? j : n - 1) - win0];
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(q8 + id * rowb + cb),
                    (__attribute__((address_space(3))) void *)(dst + i * 1024), 16, 0, 0);
            }
        };
        // helper h of 3: its k-steps of the Gram matrix of block b, into gp[h]
        auto gram = [&](int b, int h) {
            const T *R = ring(b);
            typename MF::acc acc = {T(0), T(0), T(0), T(0)};
            const int r = lane & 15, kq = lane >> 4;
            for (int ks = h * nk / 3; ks < (h + 1) * nk / 3; ++ks) {
                const int cc = 4 * ks + kq;
                const T v = cc < K ? R[r * ldq + cc] : T(0);
                acc = MF::step(v, v, acc);  // A[r][k] = B[k][r] = q_r[cc]
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) gp[h][MF::row(lane, i)][lane & 15] = acc[i];
        };
        // L of block b from the helpers' partials (thread = entry (m, t))
        auto combine = [&](int b) {
            const int m = tid >> 4, t = tid & 15;
            T v = T(0);
            if (t < m) {
                const T g = gp[0][m][t] + gp[1][m][t] + gp[2][m][t];
                v = pw[0][m - 1 - t] * hp.lr_pu * g + pw[1][m - 1 - t] * lr_bu;
            }
            lm[b & 1][m][t] = v;
        };
        // <q_m, P>_fac of block b (thread = (m, 16-lane part); DPP sums inside each row of 16)
        auto x0 = [&](int b) {
            const T *R = ring(b);
            const int m = tid >> 4, part = tid & 15;
            T acc = T(0);
            for (int cc = part; cc < K; cc += 16) acc += R[m * ldq + cc] * P[cc];
            acc += dpp<0xB1>(acc);
            acc += dpp<0x4E>(acc);
            acc += dpp<0x141>(acc);
            acc += dpp<0x140>(acc);
            if (part == 0) X0[m] = acc;
        };

        load_win(0);
        if (col) {  // P = [p_u | 1 | mu + bu | 0..]
            const T bu0 = bu[u];
            P[c] = fac ? pu[(int64_t)u * ldu + c]
                       : (c == K ? (biased ? T(1) : T(0)) : (ub ? hp.gm + bu0 : T(0)));
        }
        lds_barrier();
        if (wu == 1) {
            for (int b = 0; b < 3 && b < nb; ++b) dma(b);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_barrier();
        if (w > 0) gram(0, w - 1);
        lds_barrier();
        combine(0);
        x0(0);
        lds_barrier();
        for (int b = 0; b < nb; ++b) {
            const T *R = ring(b);
            const int len = n - b * kGB < kGB ? n - b * kGB : kGB;
            // ---- A: wave 0 solves block b; wave 1 starts block b+3's gather; waves 1-3 build
            // block b+1's Gram matrix
            if (wu == 0) {
                const int m = lane & 15;
                const int j = b * kGB + m;
                T rhs = (j < n ? rtw[j - win0] : T(0)) - pw[0][m] * X0[m] - R[m * ldq + K] * P[K] -
                        pw[1][m] * P[K + 1] - pw[2][m];
                T Lr[kGB];
#pragma unroll
                for (int t = 0; t < kGB; ++t) Lr[t] = lm[b & 1][m][t];
#pragma unroll
                for (int t = 0; t < kGB; ++t) {
                    if (t < len) {  // (L[m][t] = 0 for t >= m: lane t keeps err_t)
                        const T e = readlane(rhs, t);
                        rhs -= Lr[t] * e;
                    }
                }
                if (lane < len) E[lane] = rhs;
            } else {
                if (wu == 1 && b + 3 < nb) dma(b + 3);
                if (b + 1 < nb) gram(b + 1, w - 1);
            }
            lds_barrier();
            // ---- B: L of block b+1; the row recursion over block b (lane = column): the
            // checkpoint row p_{c+1} of every pair (c, c+1) with its two errors, the end row
            if (b + 1 < nb) combine(b + 1);
            if (col) {
                T p = P[c];
                for (int t = 0; t < len; ++t) {
                    const T e = E[t];
                    p = (apc * p + kvc) + e * (lrpc * R[t * ldq + c]);
                    if (!(t & 1)) {
                        const int64_t pair = (b * kGB + t) >> 1;
                        if (c < err_col) lrows[pair * ldq + c] = p;
                        else if (c == err_col) lrows[pair * ldq + c] = e;
                        else if (c == err_col + 1) lrows[pair * ldq + c] = t + 1 < len ? E[t + 1] : T(0);
                    }
                }
                P[c] = p;
            }
            lds_barrier();
            // ---- C: <q_m, P> of block b+1; wave 1 retires block b+2's gather (block b+3's stays
            // in flight); the next id / rating window before the blocks after b+1 need it
            if (b + 1 < nb) x0(b + 1);
            if (wu == 1 && b + 3 < nb) {
                // (vmcnt's field is 6 bits: at most 63 pieces, i.e. rows of <= 4 KiB)
                if (pieces == 13) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
                else if (pieces == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
                else if (pieces == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else if (wu == 1) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const int jn = (b + 5) * kGB;  // (block b+4's gather and the chain's ratings of b+1)
            if (jn - kGB < n && jn > win0 + kGWin) {
                lds_barrier();
                if (wu == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                load_win((b + 1) * kGB);
            }
            lds_barrier();
        }
        // the user's final row, bias and |p_u|^2 (mf.pyx:264-267; the log fold's <p^2>)
        double sq = 0;
        if (col) {
            const T p = P[c];
            if (fac) {
                pu[(int64_t)u * ldu + c] = p;
                sq = (double)p * (double)p;
            }
            if (ub) bu[u] = p - hp.gm;
        }
        sq = wave_sum(sq);
        if (lane == 0) sqw[w] = sq;
        lds_barrier();
        if (tid == 0 && psq) psq[u] = sqw[0] + sqw[1] + sqw[2] + sqw[3];
        lds_barrier();
    }
}

// ---------------------------------------------------------------- NMF
//
// NMF.sgd (matrix_factorization.pyx:646-735): within an epoch the factors are constant; every
// rating adds q_i r, q_i est to its user's numerator / denominator and p_u r, p_u est to its
// item's, then both sides take a multiplicative step.  Two race-free passes per epoch:
//   nmf_user_kernel  one wave per user: est of each rating (dot products of a 16-row batch are
//                    independent; with biases the b_u recursion is a scalar chain), the user's
//                    sums in registers, p_u's step into pu_next; est (and the item-bias step of
//                    the rating, biased) saved per CSR position;
//   nmf_item_kernel  one wave per item over its ratings (CSC order): p_u r, p_u est summed from
//                    the OLD pu, q_i's step; biased: b_i += w(N) * sum of the saved bias steps
//                    (the snapshot + count-aware rule of the delta log, oracle bias_log=1).

template <typename T, int G, bool BIASED>
__global__ __launch_bounds__(kBlock) void nmf_user_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, int n_users, const T *__restrict__ pu, T *__restrict__ pu_next,
    T *__restrict__ bu, int ldu, const T *__restrict__ qb, int ldq, int K, T reg_pu, T lr_bu,
    T reg_bu, T lr_bi, T reg_bi, T gm, T *__restrict__ est_out, T *__restrict__ blog)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    int cq[G], cu[G];
    vec fac[G];
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;
        cq[v] = c0 < ldq ? c0 : 0;  // (lanes past the row re-read column 0: no branch)
        cu[v] = c0 < ldu ? c0 : 0;
#pragma unroll
        for (int e = 0; e < W; ++e) L::set(fac[v], e, c0 + e < K ? T(1) : T(0));
    }
    // the bias column K of an item row: group, lane and element of the Lane8 layout
    const int kg = K / (kWave * W), kl = (K / W) % kWave, ke = K % W;
    const T abu = T(1) - lr_bu * reg_bu, kb = gm * (T(1) - abu);
    constexpr int kB = 16;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        if (n <= 0) continue;
        const T *prow = pu + u * (int64_t)ldu;
        vec p[G], un[G], ud[G];
#pragma unroll
        for (int v = 0; v < G; ++v) {
            p[v] = fac[v] * *(const vec *)(prow + cu[v]);
            un[v] = ud[v] = L::splat(T(0));
        }
        T cb = BIASED ? gm + bu[u] : T(0);  // mu + b_u (NMF unbiased: est = dot exactly)
        for (int x0 = 0; x0 < n; x0 += kWave) {
            const int cnt = n - x0 < kWave ? n - x0 : kWave;
            const int gi = items[s + x0 + (lane < cnt ? lane : cnt - 1)];
            const T gr = ratings[s + x0 + (lane < cnt ? lane : cnt - 1)];
            T e_l = T(0), b_l = T(0);
            for (int x = 0; x < cnt; x += kB) {
                vec q[kB][G];
                T dot[kB], bi[kB];
#pragma unroll
                for (int a = 0; a < kB; ++a) {
                    const T *qrow = qb + (int64_t)readlane(gi, x + a < cnt ? x + a : cnt - 1) * ldq;
#pragma unroll
                    for (int v = 0; v < G; ++v) q[a][v] = *(const vec *)(qrow + cq[v]);
                }
#pragma unroll
                for (int a = 0; a < kB; ++a) {  // independent reductions: interleaved by the compiler
                    vec part = L::splat(T(0));
#pragma unroll
                    for (int v = 0; v < G; ++v) part += q[a][v] * p[v];
                    dot[a] = wave_sum_u(L::hsum(part));
                    bi[a] = BIASED ? readlane(L::get(q[a][kg], ke), kl) : T(0);
                }
#pragma unroll
                for (int a = 0; a < kB; ++a) {
                    if (x + a >= cnt) break;
                    const T r = readlane(gr, x + a);
                    const T est = (cb + bi[a]) + dot[a];  // mf.pyx:703
                    const T err = r - est;
                    if (BIASED) {                          // mf.pyx:707-709
                        const T bstep = lr_bi * (err - reg_bi * bi[a]);
                        b_l = lane == x + a ? bstep : b_l;
                        cb = lr_bu * err + (abu * cb + kb);
                    }
#pragma unroll
                    for (int v = 0; v < G; ++v) {          // mf.pyx:712-716 (user side)
                        un[v] += q[a][v] * r;
                        ud[v] += q[a][v] * est;
                    }
                    e_l = lane == x + a ? est : e_l;
                }
            }
            if (lane < cnt) {
                est_out[s + x0 + lane] = e_l;
                if (BIASED) blog[s + x0 + lane] = b_l;
            }
        }
        const T nreg = (T)n * reg_pu;  // mf.pyx:719-723
        T *orow = pu_next + u * (int64_t)ldu;
#pragma unroll
        for (int v = 0; v < G; ++v) {
            const int c0 = (lane + kWave * v) * W;
            if (c0 < ldu) {
                vec o;
#pragma unroll
                for (int e = 0; e < W; ++e) {
                    const T pf = L::get(p[v], e);
                    const T den = L::get(ud[v], e) + nreg * pf;
                    L::set(o, e, c0 + e < K ? pf * (L::get(un[v], e) / den) : T(0));
                }
                *(vec *)(orow + c0) = o;
            }
        }
        if (BIASED && lane == 0) bu[u] = cb - gm;
    }
}

template <typename T, int G, bool BIASED>
__global__ __launch_bounds__(kBlock) void nmf_item_kernel(
    const int64_t *__restrict__ csc_ptr, const int64_t *__restrict__ csc_pos,
    const int32_t *__restrict__ row_user, const T *__restrict__ ratings, const T *__restrict__ est,
    const T *__restrict__ blog, const T *__restrict__ pu, int ldu, T *__restrict__ qb, int ldq,
    int K, int n_items, T reg_qi, double eta_b, int count_rule)
{
    using L = Lane8<T>;
    using vec = typename L::vec;
    constexpr int W = L::W;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    int cu[G];
#pragma unroll
    for (int v = 0; v < G; ++v) {
        const int c0 = (lane + kWave * v) * W;
        cu[v] = c0 < ldu ? c0 : 0;
    }
    constexpr int kB = 16;
    for (int64_t i = wave; i < n_items; i += n_waves) {
        const int64_t b = csc_ptr[i];
        const int N = (int)(csc_ptr[i + 1] - b);
        vec in[G], id[G];
#pragma unroll
        for (int v = 0; v < G; ++v) in[v] = id[v] = L::splat(T(0));
        T bs = T(0);
        for (int x0 = 0; x0 < N; x0 += kWave) {
            const int cnt = N - x0 < kWave ? N - x0 : kWave;
            const int64_t k = csc_pos[b + x0 + (lane < cnt ? lane : cnt - 1)];
            const int uu = row_user[k];
            const T r_l = ratings[k], e_l = est[k];
            if (BIASED && lane < cnt) bs += blog[k];
            for (int x = 0; x < cnt; x += kB) {
                vec p[kB][G];
#pragma unroll
                for (int a = 0; a < kB; ++a) {
                    const T *prow = pu + (int64_t)readlane(uu, x + a < cnt ? x + a : cnt - 1) * ldu;
#pragma unroll
                    for (int v = 0; v < G; ++v) p[a][v] = *(const vec *)(prow + cu[v]);
                }
#pragma unroll
                for (int a = 0; a < kB; ++a) {
                    if (x + a >= cnt) break;
                    const T r = readlane(r_l, x + a), e = readlane(e_l, x + a);
#pragma unroll
                    for (int v = 0; v < G; ++v) {  // mf.pyx:712-716 (item side)
                        in[v] += p[a][v] * r;
                        id[v] += p[a][v] * e;
                    }
                }
            }
        }
        const T nreg = (T)N * reg_qi;  // mf.pyx:726-730
        T *qrow = qb + i * (int64_t)ldq;
#pragma unroll
        for (int v = 0; v < G; ++v) {
            const int c0 = (lane + kWave * v) * W;
#pragma unroll
            for (int e = 0; e < W; ++e) {
                const int c = c0 + e;
                if (c < K) {
                    const T qf = qrow[c];
                    const T den = L::get(id[v], e) + nreg * qf;
                    qrow[c] = qf * (L::get(in[v], e) / den);
                }
            }
        }
        if (BIASED) {
            const T tot = wave_sum(bs);
            if (lane == 0) {
                double w = 1.0;
                if (count_rule && N > 1) w = -expm1(N * log1p(-eta_b)) / (N * eta_b);
                qrow[K] += (T)w * tot;
            }
        }
    }
}

// Small rows (NMF's default K=15: a 64-byte row) waste most of a wave in the layouts above and
// pay a 64-lane reduction per rating.  Segmented layout: the wave is R = 64/S segments of S
// lanes, E elements per lane (S E >= the row width); segment g takes rating x0 + b R + g, so one
// step gathers R rows with one load per lane and reduces R dots with log2 S shuffles.  Each
// segment keeps its own numerator / denominator; the segments are summed once per user / item.
template <int S, typename T>
__device__ __forceinline__ T seg_sum(T x) {
#pragma unroll
    for (int m = 1; m < S; m <<= 1) x += __shfl_xor(x, m, kWave);
    return x;
}
template <int S, typename T>
__device__ __forceinline__ T cross_seg_sum(T x) {
#pragma unroll
    for (int m = S; m < kWave; m <<= 1) x += __shfl_xor(x, m, kWave);
    return x;
}

// unbiased NMF user pass (mf.pyx:697-723 with biased=False: est = dot, the ratings of a user
// are independent within the epoch)
template <typename T, int S, int E>
__global__ __launch_bounds__(kBlock) void nmf_user_seg_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, int n_users, const T *__restrict__ pu, T *__restrict__ pu_next,
    int ldu, const T *__restrict__ qb, int ldq, int K, T reg_pu, T *__restrict__ est_out)
{
    constexpr int R = kWave / S, kB = 8;  // R kB ratings' rows in flight per wave
    const int lane = threadIdx.x & (kWave - 1), seg = lane / S, c0 = (lane % S) * E;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        if (n <= 0) continue;
        T p[E], un[E], ud[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            p[e] = c0 + e < K ? pu[u * ldu + c0 + e] : T(0);
            un[e] = ud[e] = T(0);
        }
        for (int x0 = 0; x0 < n; x0 += R * kB) {
            T q[kB][E], r[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int j = x0 + b * R + seg;
                const bool ok = j < n;
                const int64_t k = s + (ok ? j : n - 1);
                const T *qrow = qb + (int64_t)items[k] * ldq;
                r[b] = ratings[k];
#pragma unroll
                for (int e = 0; e < E; ++e) q[b][e] = (ok && c0 + e < ldq) ? qrow[c0 + e] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                T part = T(0);
#pragma unroll
                for (int e = 0; e < E; ++e) part += q[b][e] * p[e];
                const T est = seg_sum<S>(part);  // mf.pyx:703 (unbiased: the dot product)
#pragma unroll
                for (int e = 0; e < E; ++e) {   // mf.pyx:712-716 (user side); masked: q = 0
                    un[e] += q[b][e] * r[b];
                    ud[e] += q[b][e] * est;
                }
                const int j = x0 + b * R + seg;
                if (j < n && (lane % S) == 0) est_out[s + j] = est;
            }
        }
        const T nreg = (T)n * reg_pu;  // mf.pyx:719-723
#pragma unroll
        for (int e = 0; e < E; ++e) {
            un[e] = cross_seg_sum<S>(un[e]);
            ud[e] = cross_seg_sum<S>(ud[e]);
            const int c = c0 + e;
            if (seg == 0 && c < ldu)
                pu_next[u * ldu + c] = c < K ? p[e] * (un[e] / (ud[e] + nreg * p[e])) : T(0);
        }
    }
}

// NMF item pass (mf.pyx:712-716 item side, :726-730), biased or not
template <typename T, int S, int E, bool BIASED>
__global__ __launch_bounds__(kBlock) void nmf_item_seg_kernel(
    const int64_t *__restrict__ csc_ptr, const int64_t *__restrict__ csc_pos,
    const int32_t *__restrict__ row_user, const T *__restrict__ ratings, const T *__restrict__ est,
    const T *__restrict__ blog, const T *__restrict__ pu, int ldu, T *__restrict__ qb, int ldq,
    int K, int n_items, T reg_qi, double eta_b, int count_rule)
{
    constexpr int R = kWave / S, kB = 8;
    const int lane = threadIdx.x & (kWave - 1), seg = lane / S, c0 = (lane % S) * E;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t i = wave; i < n_items; i += n_waves) {
        const int64_t b0 = csc_ptr[i];
        const int N = (int)(csc_ptr[i + 1] - b0);
        T in[E], id[E], bs = T(0);
#pragma unroll
        for (int e = 0; e < E; ++e) in[e] = id[e] = T(0);
        for (int x0 = 0; x0 < N; x0 += R * kB) {
            T pr[kB][E], r[kB], ev[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int x = x0 + b * R + seg;
                const bool ok = x < N;
                const int64_t k = csc_pos[b0 + (ok ? x : N - 1)];
                const T *prow = pu + (int64_t)row_user[k] * ldu;
                r[b] = ratings[k];
                ev[b] = est[k];
                if (BIASED && ok && (lane % S) == 0) bs += blog[k];
#pragma unroll
                for (int e = 0; e < E; ++e) pr[b][e] = (ok && c0 + e < ldu) ? prow[c0 + e] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kB; ++b)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    in[e] += pr[b][e] * r[b];
                    id[e] += pr[b][e] * ev[b];
                }
        }
        const T nreg = (T)N * reg_qi;
        T *qrow = qb + i * (int64_t)ldq;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            in[e] = cross_seg_sum<S>(in[e]);
            id[e] = cross_seg_sum<S>(id[e]);
            const int c = c0 + e;
            if (seg == 0 && c < K) {
                const T qf = qrow[c];
                qrow[c] = qf * (in[e] / (id[e] + nreg * qf));
            }
        }
        if (BIASED) {
            const T tot = wave_sum(bs);
            if (lane == 0) {
                double w = 1.0;
                if (count_rule && N > 1) w = -expm1(N * log1p(-eta_b)) / (N * eta_b);
                qrow[K] += (T)w * tot;
            }
        }
    }
}

// The one-wave-per-item pass is bound by the most-rated item's chain of dependent gathers
// (csc_pos -> row_user -> the p_u row, ~6 us per 64 ratings).  Piece form: nmf_item_piece_kernel
// reduces each <= 64-rating piece of an item's CSC range (one wave, segmented layout) into a
// scratch row [sum p r | sum p est | sum blog]; nmf_item_fold_kernel adds an item's pieces in
// order (fixed, deterministic) and takes q_i's step.
template <typename T, int S, int E, bool BIASED>
__global__ __launch_bounds__(kBlock) void nmf_item_piece_kernel(
    const int64_t *__restrict__ csc_pos, const int32_t *__restrict__ row_user,
    const T *__restrict__ ratings, const T *__restrict__ est, const T *__restrict__ blog,
    const T *__restrict__ pu, int ldu, int ldq, const int64_t *__restrict__ piece_beg,
    int64_t n_pieces, T *__restrict__ scratch, const T *__restrict__ csc_ratings,
    const int32_t *__restrict__ csc_user)
{
    // csc_ratings / csc_user (optional): the ratings and their users already in CSC order, read
    // coalesced at CSC position b0 + x instead of gathered through k (two fewer 4-byte random
    // reads per rating, each a whole cache line); est stays gathered
    constexpr int R = kWave / S, kB = 8;
    const int lane = threadIdx.x & (kWave - 1), seg = lane / S, c0 = (lane % S) * E;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t sw = 2 * (int64_t)ldq + 1;
    for (int64_t pc = wave; pc < n_pieces; pc += n_waves) {
        const int64_t b0 = piece_beg[pc];
        const int N = (int)(piece_beg[pc + 1] - b0);  // 1 .. 64
        T in[E], id[E], bs = T(0);
#pragma unroll
        for (int e = 0; e < E; ++e) in[e] = id[e] = T(0);
        for (int x0 = 0; x0 < N; x0 += R * kB) {
            T pr[kB][E], r[kB], ev[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int x = x0 + b * R + seg;
                const bool ok = x < N;
                const int64_t xp = b0 + (ok ? x : N - 1);
                const int64_t k = csc_pos[xp];
                const T *prow = pu + (int64_t)(csc_user ? csc_user[xp] : row_user[k]) * ldu;
                r[b] = csc_ratings ? csc_ratings[xp] : ratings[k];
                ev[b] = est[k];
                if (BIASED && ok && (lane % S) == 0) bs += blog[k];
#pragma unroll
                for (int e = 0; e < E; ++e) pr[b][e] = (ok && c0 + e < ldu) ? prow[c0 + e] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kB; ++b)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    in[e] += pr[b][e] * r[b];
                    id[e] += pr[b][e] * ev[b];
                }
        }
        T *row = scratch + pc * sw;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            in[e] = cross_seg_sum<S>(in[e]);
            id[e] = cross_seg_sum<S>(id[e]);
            const int c = c0 + e;
            if (seg == 0 && c < ldq) {
                row[c] = in[e];
                row[ldq + c] = id[e];
            }
        }
        if (BIASED) {
            const T tot = wave_sum(bs);
            if (lane == 0) row[2 * ldq] = tot;
        }
    }
}

constexpr int kFoldBatch = 8;  // pieces loaded per step of a fold

template <typename T>
__global__ __launch_bounds__(kBlock) void nmf_item_fold_kernel(
    const int64_t *__restrict__ csc_ptr, const int32_t *__restrict__ item_piece_ptr, int n_items,
    const T *__restrict__ scratch, T *__restrict__ qb, int ldq, int K, T reg_qi, int biased,
    double eta_b, int count_rule)
{
    const int lane = threadIdx.x & (kWave - 1);  // lane = column (ldq <= 64 on this path)
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t sw = 2 * (int64_t)ldq + 1;
    for (int64_t i = wave; i < n_items; i += n_waves) {
        const int N = (int)(csc_ptr[i + 1] - csc_ptr[i]);
        T in = T(0), id = T(0), bs = T(0);
        const int p1 = item_piece_ptr[i + 1];
        for (int p0 = item_piece_ptr[i]; p0 < p1; p0 += kFoldBatch) {
            // kFoldBatch pieces' loads in flight, then added in piece order
            T a[kFoldBatch], d[kFoldBatch], bb[kFoldBatch];
#pragma unroll
            for (int b = 0; b < kFoldBatch; ++b) {
                const bool ok = p0 + b < p1;
                const T *row = scratch + (int64_t)(ok ? p0 + b : p0) * sw;
                a[b] = ok && lane < ldq ? row[lane] : T(0);
                d[b] = ok && lane < ldq ? row[ldq + lane] : T(0);
                bb[b] = ok && biased ? row[2 * ldq] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kFoldBatch; ++b) {
                if (p0 + b < p1) {
                    in += a[b];
                    id += d[b];
                    bs += bb[b];
                }
            }
        }
        T *qrow = qb + i * (int64_t)ldq;
        if (lane < K) {  // mf.pyx:726-730
            const T qf = qrow[lane];
            qrow[lane] = qf * (in / (id + (T)N * reg_qi * qf));
        }
        if (biased && lane == 0) {
            double w = 1.0;
            if (count_rule && N > 1) w = -expm1(N * log1p(-eta_b)) / (N * eta_b);
            qrow[K] += (T)w * bs;
        }
    }
}

// The unbiased user pass in the same piece form (its one-wave-per-user kernel is bound by the
// most-rated user's chain): nmf_user_piece_kernel takes one <= 64-rating piece of a user's CSR
// range (its owner piece_user[pc]), writes every rating's estimate and the piece's
// [sum q r | sum q est] scratch row; nmf_user_fold_kernel adds a user's pieces in order and takes
// p_u's step into pu_next (mf.pyx:697-723 with biased=False).
template <typename T, int S, int E>
__global__ __launch_bounds__(kBlock) void nmf_user_piece_kernel(
    const int32_t *__restrict__ items, const T *__restrict__ ratings,
    const T *__restrict__ pu, int ldu, const T *__restrict__ qb, int ldq, int K,
    const int64_t *__restrict__ piece_beg, const int32_t *__restrict__ piece_user,
    int64_t n_pieces, T *__restrict__ scratch, T *__restrict__ est_out)
{
    constexpr int R = kWave / S, kB = 8;
    const int lane = threadIdx.x & (kWave - 1), seg = lane / S, c0 = (lane % S) * E;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t sw = 2 * (int64_t)ldu;
    for (int64_t pc = wave; pc < n_pieces; pc += n_waves) {
        const int64_t s = piece_beg[pc];
        const int n = (int)(piece_beg[pc + 1] - s);  // 1 .. 64
        const int64_t u = piece_user[pc];
        T p[E], un[E], ud[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            p[e] = c0 + e < K ? pu[u * ldu + c0 + e] : T(0);
            un[e] = ud[e] = T(0);
        }
        for (int x0 = 0; x0 < n; x0 += R * kB) {
            T q[kB][E], r[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int j = x0 + b * R + seg;
                const bool ok = j < n;
                const int64_t k = s + (ok ? j : n - 1);
                const T *qrow = qb + (int64_t)items[k] * ldq;
                r[b] = ratings[k];
#pragma unroll
                for (int e = 0; e < E; ++e) q[b][e] = (ok && c0 + e < ldq) ? qrow[c0 + e] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                T part = T(0);
#pragma unroll
                for (int e = 0; e < E; ++e) part += q[b][e] * p[e];
                const T est = seg_sum<S>(part);  // mf.pyx:703
#pragma unroll
                for (int e = 0; e < E; ++e) {   // mf.pyx:712-716 (user side); masked: q = 0
                    un[e] += q[b][e] * r[b];
                    ud[e] += q[b][e] * est;
                }
                const int j = x0 + b * R + seg;
                if (j < n && (lane % S) == 0) est_out[s + j] = est;
            }
        }
        T *row = scratch + pc * sw;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            un[e] = cross_seg_sum<S>(un[e]);
            ud[e] = cross_seg_sum<S>(ud[e]);
            const int c = c0 + e;
            if (seg == 0 && c < ldu) {
                row[c] = un[e];
                row[ldu + c] = ud[e];
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void nmf_user_fold_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ user_piece_ptr, int n_users,
    const T *__restrict__ scratch, const T *__restrict__ pu, T *__restrict__ pu_next, int ldu,
    int K, T reg_pu)
{
    const int lane = threadIdx.x & (kWave - 1);  // lane = column (ldu <= 64 on this path)
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t sw = 2 * (int64_t)ldu;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int n = (int)(row_ptr[u + 1] - row_ptr[u]);
        if (n <= 0) continue;  // as nmf_user_seg_kernel: no rating, no step
        T un = T(0), ud = T(0);
        const int p1 = user_piece_ptr[u + 1];
        for (int p0 = user_piece_ptr[u]; p0 < p1; p0 += kFoldBatch) {
            T a[kFoldBatch], d[kFoldBatch];
#pragma unroll
            for (int b = 0; b < kFoldBatch; ++b) {
                const bool ok = p0 + b < p1 && lane < ldu;
                const T *row = scratch + (int64_t)(p0 + b < p1 ? p0 + b : p0) * sw;
                a[b] = ok ? row[lane] : T(0);
                d[b] = ok ? row[ldu + lane] : T(0);
            }
#pragma unroll
            for (int b = 0; b < kFoldBatch; ++b) {
                if (p0 + b < p1) {
                    un += a[b];
                    ud += d[b];
                }
            }
        }
        if (lane < ldu) {  // mf.pyx:719-723
            const T pf = lane < K ? pu[u * ldu + lane] : T(0);
            pu_next[u * ldu + lane] = lane < K ? pf * (un / (ud + (T)n * reg_pu * pf)) : T(0);
        }
    }
}

// the segmented layout for rows of <= 32 lanes: f(S, E); 0 when the row is too wide for it
#ifndef MF_NMF_SEG
#define MF_NMF_SEG 1
#endif
template <typename T, typename F>
int dispatch_seg(int width, F &&f) {
    constexpr int E = sizeof(T) == 4 ? 2 : 1;
    using E_c = std::integral_constant<int, E>;
    if (!MF_NMF_SEG) return -1;
    if (width <= 4 * E) return f(std::integral_constant<int, 4>{}, E_c{});
    if (width <= 8 * E) return f(std::integral_constant<int, 8>{}, E_c{});
    if (width <= 16 * E) return f(std::integral_constant<int, 16>{}, E_c{});
    if (width <= 32 * E) return f(std::integral_constant<int, 32>{}, E_c{});
    return -1;
}

// ---------------------------------------------------------------- baseline ALS (8(f) 4)
//
// baseline_als (optimize_baselines.pyx:14-54): per epoch every item's bias from the current user
// biases, then every user's bias from the new item biases.  One wave per item / user, lanes
// over its ratings, one wave sum.
constexpr int kAlsBatch = 8;  // strides of 64 ratings whose loads are issued together

template <typename T>
__global__ __launch_bounds__(kBlock) void als_item_kernel(
    const int64_t *__restrict__ csc_ptr, const int64_t *__restrict__ csc_pos,
    const int32_t *__restrict__ row_user, const T *__restrict__ ratings, const T *__restrict__ bu,
    T *__restrict__ bi, int n_items, T gm, T reg_i, const T *__restrict__ csc_ratings,
    const int32_t *__restrict__ csc_user)
{
    // csc_ratings / csc_user (optional): CSC-ordered copies, read coalesced (no csc_pos hop)
    const bool direct = csc_ratings && csc_user;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t i = wave; i < n_items; i += n_waves) {
        const int64_t b = csc_ptr[i];
        const int N = (int)(csc_ptr[i + 1] - b);
        T dev = T(0);
        for (int x0 = lane; x0 < N; x0 += kAlsBatch * kWave) {
            // kAlsBatch strides' gather chains (csc_pos -> row_user -> bu) in flight, then
            // added in the lane's x order (the same sums as one stride at a time)
            T t[kAlsBatch];
            if (direct) {
#pragma unroll
                for (int j = 0; j < kAlsBatch; ++j) {
                    const int x = x0 + j * kWave;
                    const int64_t xp = b + (x < N ? x : N - 1);
                    t[j] = csc_ratings[xp] - gm - bu[csc_user[xp]];  // :43-44
                }
            } else {
                int64_t k[kAlsBatch];
#pragma unroll
                for (int j = 0; j < kAlsBatch; ++j) {
                    const int x = x0 + j * kWave;
                    k[j] = csc_pos[b + (x < N ? x : N - 1)];
                }
#pragma unroll
                for (int j = 0; j < kAlsBatch; ++j) t[j] = ratings[k[j]] - gm - bu[row_user[k[j]]];
            }
#pragma unroll
            for (int j = 0; j < kAlsBatch; ++j)
                if (x0 + j * kWave < N) dev += t[j];
        }
        dev = wave_sum(dev);
        if (lane == 0) bi[i] = dev / (reg_i + (T)N);  // :46
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void als_user_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const T *__restrict__ bi, T *__restrict__ bu, int n_users, T gm,
    T reg_u)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int64_t s = row_ptr[u];
        const int n = (int)(row_ptr[u + 1] - s);
        T dev = T(0);
        for (int x0 = lane; x0 < n; x0 += kAlsBatch * kWave) {
            T t[kAlsBatch];
#pragma unroll
            for (int j = 0; j < kAlsBatch; ++j) {
                const int64_t x = s + (x0 + j * kWave < n ? x0 + j * kWave : n - 1);
                t[j] = ratings[x] - gm - bi[items[x]];  // :50-51
            }
#pragma unroll
            for (int j = 0; j < kAlsBatch; ++j)
                if (x0 + j * kWave < n) dev += t[j];
        }
        dev = wave_sum(dev);
        if (lane == 0) bu[u] = dev / (reg_u + (T)n);  // :52
    }
}

// ---------------------------------------------------------------- inference

// ---------------------------------------------------------------- SVD++ deferred y update
//
// With one wave per user every user of an epoch-chunk gathers the chunk-start y_j anyway; its
// end-of-user update is the affine map y_j <- A_u y_j + c_u (A_u = (1 - lr_yj reg_yj)^{|I_u|}),
// which the atomic schedule applies with float atomics in whatever order users finish.
// Deferred form: the epoch kernel stores c_u (ycbuf[u]); after the chunk the maps of the chunk's
// users that rated j are composed in CSR (user) order -- race-free, deterministic, no atomics.
// (Summing the c_u and applying prod A_u once diverges: on a popular item prod A_u ~ e^-80, the
// early users' c_u must decay with the later users' factors.)  Affine maps compose associatively,
// (A2, c2) o (A1, c1) = (A2 A1, A2 c1 + c2), so the composition is a two-level tree over the log's
// pieces (<= 64 ratings of one item): y_piece_kernel composes each piece (one wave, one FMA per
// user, two groups of 8 users' rows in flight), y_apply_kernel applies an item's pieces in order.
#ifndef MF_YFOLD_U
#define MF_YFOLD_U 8
#endif
template <typename T, int V>
__global__ __launch_bounds__(kBlock) void y_piece_kernel(
    int ldu, int K, const T *__restrict__ ycbuf, const T *__restrict__ uA,
    const int32_t *__restrict__ item_users, const int32_t *__restrict__ piece_beg,
    int64_t n_pieces, T *__restrict__ pc_c, T *__restrict__ pc_A,
    const int32_t *__restrict__ piece_item, const int32_t *__restrict__ item_piece_ptr,
    T *__restrict__ yj)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t pc = wave; pc < n_pieces; pc += n_waves) {
        const int b = piece_beg[pc], e = piece_beg[pc + 1];
        const int my_u = item_users[b + (lane < e - b ? lane : e - b - 1)];  // lane x: user x
        T cacc[V], Aacc = T(1);
#pragma unroll
        for (int v = 0; v < V; ++v) cacc[v] = T(0);
        constexpr int kU = MF_YFOLD_U;  // users' rows per group, two groups in flight
        const int n = e - b;
        auto load = [&](const int x, T (&g)[kU][V], T (&A)[kU]) {
#pragma unroll
            for (int a = 0; a < kU; ++a) {
                const bool ok = x + a < n;
                const int64_t u = readlane(my_u, ok ? x + a : 0);
                A[a] = ok ? uA[u] : T(1);  // (past the piece: the identity map)
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const int c = lane + kWave * v;
                    g[a][v] = (ok && c < K) ? ycbuf[u * ldu + c] : T(0);
                }
            }
        };
        auto comp = [&](T (&g)[kU][V], T (&A)[kU]) {
#pragma unroll
            for (int a = 0; a < kU; ++a) {
                Aacc = A[a] * Aacc;
#pragma unroll
                for (int v = 0; v < V; ++v) cacc[v] = A[a] * cacc[v] + g[a][v];
            }
        };
        T gA[kU][V], AA[kU], gB[kU][V], AB[kU];
        load(0, gA, AA);
        for (int x = 0; x < n; x += 2 * kU) {
            if (x + kU < n) load(x + kU, gB, AB);
            comp(gA, AA);
            if (x + kU >= n) break;
            if (x + 2 * kU < n) load(x + 2 * kU, gA, AA);
            comp(gB, AB);
        }
        if (piece_item) {  // the item's only piece: its map applied to y_j here (y_apply skips it)
            const int j = piece_item[pc];
            if (item_piece_ptr[j + 1] - item_piece_ptr[j] == 1) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const int c = lane + kWave * v;
                    if (c < K) yj[(int64_t)j * ldu + c] = Aacc * yj[(int64_t)j * ldu + c] + cacc[v];
                }
                continue;
            }
        }
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int c = lane + kWave * v;
            if (c < ldu) pc_c[pc * ldu + c] = cacc[v];
        }
        if (lane == 0) pc_A[pc] = Aacc;
    }
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void y_apply_kernel(
    T *__restrict__ yj, int ldu, int K, const int32_t *__restrict__ item_piece_ptr, int n_items,
    const T *__restrict__ pc_c, const T *__restrict__ pc_A, int min_pieces)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t j = wave; j < n_items; j += n_waves) {
        const int p0 = item_piece_ptr[j], p1 = item_piece_ptr[j + 1];
        if (p1 - p0 < min_pieces) continue;  // (none, or -- fused -- the one y_piece applied)
        T y[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int c = lane + kWave * v;
            y[v] = c < K ? yj[j * ldu + c] : T(0);
        }
        constexpr int kP = 8;  // pieces' rows in flight (a popular item has ~60 pieces)
        for (int p = p0; p < p1; p += kP) {
            T A[kP], g[kP][V];
#pragma unroll
            for (int a = 0; a < kP; ++a) {
                const bool ok = p + a < p1;
                A[a] = ok ? pc_A[p + a] : T(1);  // (past the item: the identity map)
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const int c = lane + kWave * v;
                    g[a][v] = ok && c < K ? pc_c[(int64_t)(p + a) * ldu + c] : T(0);
                }
            }
#pragma unroll
            for (int a = 0; a < kP; ++a)  // composed in piece order
#pragma unroll
                for (int v = 0; v < V; ++v) y[v] = A[a] * y[v] + g[a][v];
        }
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int c = lane + kWave * v;
            if (c < K) yj[j * ldu + c] = y[v];
        }
    }
}

// ---------------------------------------------------------------- SVD++ q log: the fused fold
//
// One rank's fold of an SVD++ q-log chunk (mf_svdpp_qlog_fold) in ONE pass over the items, each
// item by one wave: (1) its logged q / b gradient rows (the chunk's rows of the item: positions
// item_row_beg[i] .. item_row_beg[i+1] of perm, users in order) summed with their recency weights
// (1 - eta)^(N - 1 - pos) (log_reduce_kernel's weights), then q += lr (S - w N reg q) -- what
// mf_log_reduce + mf_log_apply compute; (2) its y row composed with the chunk's users' affine
// maps y <- A_u y + c_u in CSR order (the raters of the same positions, item_users) -- what
// mf_svdpp_y_fold computes.  Nothing round-trips through piece sums; every load is a row gather
// whose indices come from ONE coalesced vector load per 64 rows, so a wave keeps kF rows in
// flight per part and the launch's occupancy (kFoldWPC waves per CU) hides the rest of the
// latency.  Items the chunk did not touch are skipped (their rows do not change).  Block 0: the
// next chunk's {sum |p_u|^2, count} from user_sq, like mf_log_apply's.
constexpr int kFoldF = 8;      // rows of one part in flight per wave
constexpr int kFoldWPC = 32;   // waves per CU
template <typename T, int VQ, int VY>
__global__ __launch_bounds__(kBlock) void qlog_fold_kernel(
    T *__restrict__ qb, int ldq, int K, T *__restrict__ yj, int ldu, const T *__restrict__ qlog,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ item_row_beg,
    const int32_t *__restrict__ totals, Recency rc, double lr_f, double reg_f, double lr_b,
    double reg_b, const T *__restrict__ ycbuf, const T *__restrict__ uA,
    const int32_t *__restrict__ item_users, int n_items, double *__restrict__ stat_next,
    const double *__restrict__ user_sq, int64_t n_sq, int sq_cols, const T *__restrict__ hot_sums,
    const int32_t *__restrict__ hot_item_piece_ptr, const T *__restrict__ hot_pc_c,
    const T *__restrict__ hot_pc_A)
{
    if (stat_next && blockIdx.x == 0) {
        if (user_sq) block_sum_sq(user_sq, n_sq, sq_cols, stat_next);
        else if (threadIdx.x < 2) stat_next[threadIdx.x] = 0.0;
        return;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int blk0 = stat_next ? 1 : 0;
    const int64_t wave = (int64_t)(blockIdx.x - blk0) * (kBlock / kWave) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t n_waves = ((int64_t)(gridDim.x - blk0) * kBlock) / kWave;
    double l_q, l_b;
    recency_logs(rc, l_q, l_b);
    const double n_p2 = rc.p2stat[1];
    const double eta_f = rc.lr_qi * ((n_p2 > 0 ? rc.p2stat[0] / n_p2 : 0.0) + rc.reg_qi);
    const double eta_b = rc.eta_b;
    // items in batches of 64, batch b = items b + NB t (t < 64): the most-rated (lowest-id)
    // items land in different batches, so no wave takes several hot items in a row
    const int64_t NB = (n_items + kWave - 1) / kWave;
    for (int64_t b = wave; b < NB; b += n_waves) {
        // lane t: item b + NB t's cold row range (one piece: <= 64 rows), hot piece range, N
        const int64_t it_l = b + NB * lane;
        const bool in_l = it_l < n_items;
        const int r0_l = in_l ? item_row_beg[it_l] : 0, r1_l = in_l ? item_row_beg[it_l + 1] : 0;
        const int h0_l = in_l && hot_item_piece_ptr ? hot_item_piece_ptr[it_l] : 0;
        const int h1_l = in_l && hot_item_piece_ptr ? hot_item_piece_ptr[it_l + 1] : 0;
        const int N_l = in_l ? totals[it_l] : 0;
        // the cold rows' indices of item t (lane x: row x) are loaded two items ahead of its
        // gathers, its weights and A_u one item ahead: the A_u gather and the weights need the
        // indices, so issuing all three at once stalls every item on two dependent round trips
        auto iload = [&](const int t, int &k_l, int &u_l, int &p_l) {
            const int r0 = readlane(r0_l, t), cnt = readlane(r1_l, t) - r0;
            const int xl = r0 + (lane < cnt ? lane : (cnt > 0 ? cnt - 1 : 0));
            k_l = cnt > 0 ? perm[xl] : 0;
            u_l = cnt > 0 ? item_users[xl] : 0;
            p_l = cnt > 0 ? rc.rpos[xl] : 0;
        };
        auto wload = [&](const int t, const int u_l, const int p_l, T &wf_l, T &wb_l, T &A_l) {
            const int cnt = readlane(r1_l, t) - readlane(r0_l, t);
            const int N = readlane(N_l, t);
            const bool ok = lane < cnt;
            if constexpr (sizeof(T) == 4) {  // (fp32 weights: the float exp, ~8x cheaper)
                const float back = (float)(N - 1 - p_l);
                wf_l = ok ? expf(back * (float)l_q) : 0.f;
                wb_l = ok ? expf(back * (float)l_b) : 0.f;
            } else {
                const double back = (double)(N - 1 - p_l);
                wf_l = ok ? (T)exp(back * l_q) : T(0);
                wb_l = ok ? (T)exp(back * l_b) : T(0);
            }
            A_l = cnt > 0 ? uA[u_l] : T(1);
        };
        int k_c = 0, u_c = 0, p_c = 0, k_n = 0, u_n = 0, p_n = 0;
        T wf_c, wb_c, A_c;
        iload(0, k_c, u_c, p_c);
        if (b + NB < n_items) iload(1, k_n, u_n, p_n);
        wload(0, u_c, p_c, wf_c, wb_c, A_c);
        for (int t = 0; t < kWave; ++t) {
            const int64_t i = b + NB * t;
            if (i >= n_items) break;  // (uniform)
            int k_nn = 0, u_nn = 0, p_nn = 0;
            if (t + 2 < kWave && i + 2 * NB < n_items) iload(t + 2, k_nn, u_nn, p_nn);
            T wf_n = T(0), wb_n = T(0), A_n = T(1);
            if (t + 1 < kWave && i + NB < n_items) wload(t + 1, u_n, p_n, wf_n, wb_n, A_n);
            const int cnt = readlane(r1_l, t) - readlane(r0_l, t);
            const int h0 = readlane(h0_l, t), h1 = readlane(h1_l, t);
            if (cnt > 0 || h0 < h1) {
                const int N = readlane(N_l, t);
                T q[VQ], y[VY], acc[VQ];
#pragma unroll
                for (int v = 0; v < VQ; ++v) {
                    const int c = lane + kWave * v;
                    q[v] = c < ldq ? qb[i * ldq + c] : T(0);
                    acc[v] = T(0);
                }
#pragma unroll
                for (int v = 0; v < VY; ++v) {
                    const int c = lane + kWave * v;
                    y[v] = c < K ? yj[i * ldu + c] : T(0);
                }
                // (1 + 2) a cold item: its gradient rows and its raters' c_u rows together,
                // kFoldF of each in flight
                for (int a0 = 0; a0 < cnt; a0 += kFoldF) {
                    T g[kFoldF][VQ], gy[kFoldF][VY];
#pragma unroll
                    for (int a = 0; a < kFoldF; ++a) {
                        const int x = a0 + a < cnt ? a0 + a : cnt - 1;
                        const T *row = qlog + (int64_t)readlane(k_c, x) * ldq;
                        const T *yrow = ycbuf + (int64_t)readlane(u_c, x) * ldu;
#pragma unroll
                        for (int v = 0; v < VQ; ++v) {
                            const int c = lane + kWave * v;
                            g[a][v] = c <= K ? row[c] : T(0);
                        }
#pragma unroll
                        for (int v = 0; v < VY; ++v) {
                            const int c = lane + kWave * v;
                            gy[a][v] = c < K ? yrow[c] : T(0);
                        }
                    }
#pragma unroll
                    for (int a = 0; a < kFoldF; ++a) {
                        const int x = a0 + a < kWave ? a0 + a : kWave - 1;
                        const T wf = readlane(wf_c, x), wb = readlane(wb_c, x);  // (0 past cnt)
#pragma unroll
                        for (int v = 0; v < VQ; ++v)
                            acc[v] += (lane + kWave * v == K ? wb : wf) * g[a][v];
                    }
#pragma unroll
                    for (int a = 0; a < kFoldF; ++a) {
                        if (a0 + a >= cnt) break;  // (uniform)
                        const T A = readlane(A_c, a0 + a);
#pragma unroll
                        for (int v = 0; v < VY; ++v) y[v] = A * y[v] + gy[a][v];
                    }
                }
                // (1' + 2') a hot item: its pieces' weighted sums and composed maps, in order
                for (int p0 = h0; p0 < h1; p0 += kFoldF) {
                    T g[kFoldF][VQ], gy[kFoldF][VY], A[kFoldF];
#pragma unroll
                    for (int a = 0; a < kFoldF; ++a) {
                        const bool ok = p0 + a < h1;
                        const int64_t p = ok ? p0 + a : h0;
                        A[a] = ok ? hot_pc_A[p] : T(1);  // (past the item: the identity map)
#pragma unroll
                        for (int v = 0; v < VQ; ++v) {
                            const int c = lane + kWave * v;
                            g[a][v] = ok && c <= K ? hot_sums[p * ldq + c] : T(0);
                        }
#pragma unroll
                        for (int v = 0; v < VY; ++v) {
                            const int c = lane + kWave * v;
                            gy[a][v] = ok && c < K ? hot_pc_c[p * ldu + c] : T(0);
                        }
                    }
#pragma unroll
                    for (int a = 0; a < kFoldF; ++a) {
#pragma unroll
                        for (int v = 0; v < VQ; ++v) acc[v] += g[a][v];
#pragma unroll
                        for (int v = 0; v < VY; ++v) y[v] = A[a] * y[v] + gy[a][v];
                    }
                }
                // q += lr (S - w N reg q), w N = sum_k (1 - eta)^(N-1-k) (mf_log_apply's rule)
                const double wn_f = N > 1 ? -expm1(N * l_q) / eta_f : (double)N;
                const double wn_b = N > 1 ? -expm1(N * l_b) / eta_b : (double)N;
#pragma unroll
                for (int v = 0; v < VQ; ++v) {
                    const int c = lane + kWave * v;
                    if (c <= K) {
                        const bool bc = c == K;
                        qb[i * ldq + c] = q[v] + (T)(bc ? lr_b : lr_f) *
                                                     (acc[v] - (T)(bc ? wn_b : wn_f) *
                                                                   (T)(bc ? reg_b : reg_f) * q[v]);
                    }
                }
#pragma unroll
                for (int v = 0; v < VY; ++v) {
                    const int c = lane + kWave * v;
                    if (c < K) yj[i * ldu + c] = y[v];
                }
            }
            k_c = k_n;
            u_c = u_n;
            wf_c = wf_n;
            wb_c = wb_n;
            A_c = A_n;
            k_n = k_nn;
            u_n = u_nn;
            p_n = p_nn;
        }
    }
}

// accuracy.rmse / mae over the batched estimates (algo_base.py:148-169 finishing, accuracy.py:
// 22-90): est -> fallback where impossible, minus the reader offset, clipped to the rating scale,
// against r - offset; out[0] += sum err^2, out[1] += sum |err|, out[2] += count (fp64).
template <typename T>  // (est in the model's dtype; the true ratings always fp64, as r_ui is)
__global__ __launch_bounds__(kBlock) void rating_errors_kernel(
    int64_t n, const T *__restrict__ est, const int32_t *__restrict__ impossible,
    const double *__restrict__ r, double fallback, double offset, double lo, double hi,
    double *__restrict__ out)
{
    __shared__ double part[2][kBlock / kWave];
    double se = 0, ae = 0;
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * kBlock) {
        double e = (impossible && impossible[x]) ? fallback : (double)est[x];
        e -= offset;
        e = e < lo ? lo : (e > hi ? hi : e);  // (NaN -> hi, as np.fmax(lo, np.fmin(hi, e)))
        e = e == e ? e : hi;
        const double d = (r[x] - offset) - e;
        se += d * d;
        ae += d < 0 ? -d : d;
    }
    se = wave_sum(se);
    ae = wave_sum(ae);
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        part[0][w] = se;
        part[1][w] = ae;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0, b = 0;
        for (int v = 0; v < kBlock / kWave; ++v) {
            a += part[0][v];
            b += part[1][v];
        }
        atomicAdd(out, a);
        atomicAdd(out + 1, b);
        if (blockIdx.x == 0) atomicAdd(out + 2, (double)n);
    }
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void predict_kernel(
    int64_t n, const int32_t *__restrict__ uu, const int32_t *__restrict__ ii,
    const T *__restrict__ pu, const T *__restrict__ bu, int ldu, const T *__restrict__ qb,
    int ldq, const T *__restrict__ imp, int K, int biased, T gm, T *__restrict__ est,
    int32_t *__restrict__ impossible)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t x = wave; x < n; x += n_waves) {
        const int u = uu[x], i = ii[x];
        const bool ku = u >= 0, ki = i >= 0;
        T part = T(0);
        if (ku && ki) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int f = lane + kWave * v;
                if (f < K) {
                    T pf = pu[(int64_t)u * ldu + f];
                    if (imp) pf += imp[(int64_t)u * ldu + f];
                    part += qb[(int64_t)i * ldq + f] * pf;
                }
            }
        }
        const T dot = wave_sum(part);
        if (lane == 0) {
            int bad = 0;
            T e;
            if (biased) {  // mf.pyx:283-293 / :510-521
                e = gm;
                if (ku) e += bu[u];
                if (ki) e += qb[(int64_t)i * ldq + K];
                if (ku && ki) e += dot;
            } else if (ku && ki) {
                e = dot;
            } else {  // PredictionImpossible (mf.pyx:295-296)
                e = T(0);
                bad = 1;
            }
            est[x] = e;
            impossible[x] = bad;
        }
    }
}

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void user_implicit_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items, int n_users,
    const T *__restrict__ yj, int ldu, T *__restrict__ imp, int K)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int64_t s = row_ptr[u], e = row_ptr[u + 1];
        T acc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = T(0);
        for (int64_t k = s; k < e; ++k) {  // sum(yj[j] for j in ur[u]) in ur order (mf.pyx:518)
            const T *row = yj + (int64_t)items[k] * ldu + lane;
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (lane + kWave * v < K) acc[v] += row[kWave * v];
        }
        const T sq = sqrt(T(e - s));
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int f = lane + kWave * v;
            if (f < ldu) imp[u * ldu + f] = (e > s && f < K) ? acc[v] / sq : T(0);
        }
    }
}

__global__ void xcc_selftest_kernel(int32_t *out, int n_blocks)
{
    if (threadIdx.x == 0 && (int)blockIdx.x < n_blocks) out[blockIdx.x] = xcc_id();
}

template <typename T>
__global__ void wave_sum_selftest_kernel(const T *in, T *out, int n_waves)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int w = (blockIdx.x * kBlock + threadIdx.x) / kWave;
    T v = w < n_waves ? in[(int64_t)w * kWave + lane] : T(0);
    v = wave_sum(v);
    if (w < n_waves && lane == 0) out[w] = v;
}

// ---------------------------------------------------------------- launch helpers

int n_cus() {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            n_cu = prop.multiProcessorCount;
        if (n_cu <= 0) n_cu = 256;
    }
    return n_cu;
}

// The dispatch layout the XCD masks assume (wave_slot): 8 XCDs, workgroup b on XCD
// (x0 + b) mod 8 for some x0 of the launch.
// Checked once per device with the XCC_ID register (xcc_selftest_kernel); a launch with an XCD
// mask is refused where it does not hold (e.g. a partitioned device): its waves would otherwise
// exit or share user slots, silently training some users twice and others never.
int xcd_layout_ok()
{
    static std::mutex mu;
    static int state[64] = {};  // per device: 0 unknown, 1 verified, -1 not this layout
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    std::lock_guard<std::mutex> lock(mu);
    if (state[dev] == 0) {
        constexpr int kN = 512;
        int32_t *d = nullptr, h[kN];
        bool ok = n_cus() % 8 == 0 && hipMalloc((void **)&d, sizeof(h)) == hipSuccess;
        if (ok) {
            // on an idle device (work of other streams drained first), twice: a layout that is
            // not round-robin fails both times, a transient one once
            (void)hipDeviceSynchronize();
            bool seen = false;
            for (int attempt = 0; attempt < 2 && !seen; ++attempt) {
                hipLaunchKernelGGL(xcc_selftest_kernel, dim3(kN), dim3(kWave), 0,
                                   (hipStream_t)0, d, kN);
                bool run = hipGetLastError() == hipSuccess &&
                           hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
                // (round-robin from whichever XCD the dispatcher's pointer is at: measured
                // starting at XCD 5 after earlier launches -- wave_slot only needs every 8
                // consecutive workgroups on 8 distinct XCDs)
                seen = run && h[0] >= 0 && h[0] < 8;
                for (int b = 0; seen && b < kN; ++b) seen = h[b] == (h[0] + b) % 8;
            }
            ok = seen;
            (void)hipFree(d);
        }
        state[dev] = ok ? 1 : -1;
    }
    return state[dev] > 0;
}

int check_xmask(int xmask)
{
    if ((xmask & 0xFF) && !xcd_layout_ok())
        return set_err(MF_E_UNSUPPORTED, "XCD masks need 8 XCDs dealt workgroups round-robin "
                                         "(mf_xcd_layout)");
    return 0;
}

// Default grid: enough waves to hold every scheduled user, capped at 16 waves per CU.
int64_t default_waves(int64_t n_sched) {
    const int64_t cap = (int64_t)n_cus() * 16;
    return n_sched < cap ? n_sched : cap;
}

// V = elements per lane = ceil(ld / 64)
template <typename T, typename F>
int dispatch_v(int ld, F &&f)
{
    const int v = (ld + kWave - 1) / kWave;
    if (v <= 1) return f(std::integral_constant<int, 1>{});
    if (v <= 2) return f(std::integral_constant<int, 2>{});
    if (v <= 3) return f(std::integral_constant<int, 3>{});
    if (v <= 4) return f(std::integral_constant<int, 4>{});
    if constexpr (sizeof(T) == 4) {
        if (v <= 6) return f(std::integral_constant<int, 6>{});
        if (v <= 9) return f(std::integral_constant<int, 9>{});
    } else {
        if (v <= 5) return f(std::integral_constant<int, 5>{});
    }
    return set_err(MF_E_ARG, "n_factors/ld too large");
}

int check_epoch(const mf_csr_t *c, const int32_t *sched, const void *pu, const void *bu,
                const void *qb, const mf_hyper_t *hp, int K, int ldu, int ldq, int mode,
                const void *qlog, int dtype)
{
    if (!c || !c->row_ptr || !c->items || !c->ratings) return set_err(MF_E_ARG, "null csr");
    if (!sched || !pu || !bu || !qb || !hp) return set_err(MF_E_ARG, "null argument");
    if (dtype != MF_F32 && dtype != MF_F64) return set_err(MF_E_ARG, "bad dtype");
    const int maxk = dtype == MF_F32 ? MF_MAX_FACTORS_F32 : MF_MAX_FACTORS_F64;
    if (K < 0 || K > maxk) return set_err(MF_E_ARG, "n_factors out of range");
    if (ldu < K || ldq < K + 1) return set_err(MF_E_ARG, "need ldu >= n_factors, ldq >= n_factors+1");
    if (mode < MF_MODE_PLAIN || mode > MF_MODE_LOG) return set_err(MF_E_ARG, "bad mode");
    if (mode == MF_MODE_LOG && !qlog) return set_err(MF_E_ARG, "MF_MODE_LOG needs qlog");
    const size_t esz = dtype == MF_F32 ? 4 : 8;
    if ((uint64_t)c->n_items * (uint64_t)ldq * esz >= kMaxTable ||
        (uint64_t)c->n_items * (uint64_t)ldu * esz >= kMaxTable)
        return set_err(MF_E_UNSUPPORTED, "item table >= 2 GiB (32-bit buffer offsets)");
    return 0;
}

// First of the two padding columns that hold a checkpoint row's errors (MF_EPOCH_ERR_IN_ROW):
// past the item-bias column K and the user-bias column K + 1, 8-byte aligned for fp32 (one
// lane's pair); 0 if the row has no room.
int err_column(int K, int ldq, int dtype)
{
    const int c = dtype == MF_F32 ? ((K + 3) & ~1) : K + 2;
    return c + 2 <= ldq ? c : 0;
}

// MF_EPOCH_CKPT_NARROW: the checkpoint rows' stride, K rounded up to 8 bytes (whole lane pairs)
int ckpt_narrow_ld(int K, int dtype) { return dtype == MF_F32 ? (K + 1) & ~1 : K; }

// the kernels' recency inputs (rec NULL: off)
int make_recency(const mf_recency_t *rec, const mf_hyper_t *hp, Recency &rc)
{
    rc = Recency{};
    if (!rec) return 0;
    if (!rec->rpos || !rec->totals || !rec->p2stat || !hp)
        return set_err(MF_E_ARG, "recency weights need rpos, totals, p2stat and hp");
    rc = Recency{rec->rpos, rec->pos0, rec->totals, rec->p2stat, hp->lr_qi, hp->reg_qi,
                 hp->lr_bi * (1.0 + hp->reg_bi)};
    return 0;
}

template <bool PP>
int launch_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                 int32_t ldu, void *qb, int32_t ldq, void *yj, void *qlog, void *elog, int32_t K,
                 int32_t biased, const mf_hyper_t *hp, int32_t mode, int32_t n_waves, int32_t flags,
                 int32_t dtype, void *stream, double *psq = nullptr, int32_t *status = nullptr,
                 const uint8_t *hot = nullptr, const int64_t *urow = nullptr,
                 const int32_t *crow = nullptr)
{
    const bool dups = flags & MF_EPOCH_DUP_ITEMS;
    // helper waves per chain: 3, or 1 (MF_EPOCH_SVDPP_ONE_HELPER); 0 = no helper-wave launch
    const int hx = !(flags & MF_EPOCH_SVDPP_HELPERS) ? 0
                   : (flags & MF_EPOCH_SVDPP_ONE_HELPER) ? 1 : kHxHelpers;
    if ((flags & MF_EPOCH_SVDPP_ONE_HELPER) && !hx)
        return set_err(MF_E_ARG, "MF_EPOCH_SVDPP_ONE_HELPER: with MF_EPOCH_SVDPP_HELPERS only");
    const int xmask = (flags >> MF_EPOCH_XCD_SHIFT) & 0xFF;
    if (int rc = check_epoch(csr, sched, pu, bu, qb, hp, K, ldu, ldq, mode, qlog, dtype)) return rc;
    if (int rc = check_xmask(xmask)) return rc;
    int err_col = 0;
    if (flags & MF_EPOCH_ERR_IN_ROW) {
        if (PP || mode != MF_MODE_LOG || !elog)
            return set_err(MF_E_ARG, "MF_EPOCH_ERR_IN_ROW: the SVD checkpoint log only");
        err_col = err_column(K, ldq, dtype);
        if (err_col <= 0) return set_err(MF_E_UNSUPPORTED, "MF_EPOCH_ERR_IN_ROW: no spare columns");
    }
    int ck_ld = ldq;  // the checkpoint rows' stride
    if (flags & MF_EPOCH_CKPT_NARROW) {
        if (PP || mode != MF_MODE_LOG || !elog || err_col || K < 1)
            return set_err(MF_E_ARG, "MF_EPOCH_CKPT_NARROW: the SVD checkpoint log, errors in elog");
        ck_ld = ckpt_narrow_ld(K, dtype);
    }
    if (PP && !yj) return set_err(MF_E_ARG, "null yj");
    // hot-row replicas: the range covers 2 n_items rows and the masked offsets (row + range) must
    // stay below 2^32
    if (hot && 3.0 * csr->n_items * ldq * (dtype == MF_F32 ? 4.0 : 8.0) >= 4294967296.0)
        return set_err(MF_E_UNSUPPORTED, "hot-row replicas: item table >= 1.33 GiB");
    if (n_sched <= 0) return 0;
    // default: one wave per user up to MF_EPOCH_WPC waves per CU (then strided): a wave that
    // finishes its user exits and the dispatcher starts the next one -- measured 5 us faster at
    // ML-1M than 16 waves/CU taking users in turn (the longest chains start together either way)
    const int64_t cap = (int64_t)n_cus() * MF_EPOCH_WPC;
    const int64_t waves = n_waves > 0 ? n_waves : (n_sched < cap ? n_sched : cap);
    auto run = [&](auto tag_t, auto mode_c) -> int {
        using T = decltype(tag_t);
        constexpr int M = decltype(mode_c)::value;
        return mf_ext::launch_epoch_tm<T, M, PP>(csr, sched, n_sched, pu, bu, ldu, qb, ldq, yj,
                                                  qlog, elog, K, biased, hp, waves, dups, xmask,
                                                  hx, psq, err_col, ck_ld, status, hot, urow,
                                                  (flags & MF_EPOCH_LOG_NT) != 0, crow, stream);
    };
    auto by_mode = [&](auto tag_t) -> int {
        switch (mode) {
            case MF_MODE_PLAIN: return run(tag_t, std::integral_constant<int, kPlain>{});
            case MF_MODE_ATOMIC: return run(tag_t, std::integral_constant<int, kAtomic>{});
            default: return run(tag_t, std::integral_constant<int, kLog>{});
        }
    };
    return dtype == MF_F32 ? by_mode(float{}) : by_mode(double{});
}

// hipLaunchKernelGGL, or -- after mf_launch_event(ev) on this thread -- the same launch with ev
// bound to the dispatch as its stop event (hipExtLaunchKernelGGL): ev completes with the kernel,
// no marker packet follows it in the queue (a marker costs the next kernel ~7 us of queue time)
// The pending event is taken at the entry point (StopEvent); an entry point that returns without
// launching records it on its stream instead, so "ev completes after the call's work" holds.
struct StopEvent {
    hipEvent_t ev;
    hipStream_t st;
    explicit StopEvent(void *stream) : ev(mf_ext::g_stop_event), st((hipStream_t)stream) { mf_ext::g_stop_event = nullptr; }
    ~StopEvent() { if (ev) (void)hipEventRecord(ev, st); }
    hipEvent_t take() { hipEvent_t e = ev; ev = nullptr; return e; }
};

template <typename F, typename... Args>
void launch_ev(hipEvent_t ev, F kernel, dim3 grid, dim3 block, hipStream_t st, Args... args) {
    if (ev)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, st, nullptr, ev, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
}

int elementwise_grid(int64_t total) {
    int64_t b = (total + kBlock - 1) / kBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace

extern "C" {

int mf_version(void) { return 936; }

#ifndef MF_SOURCE_HASH
#define MF_SOURCE_HASH "unknown"
#endif
// sha256 of this file, include/surprise_amd.h and the compile lines (surprise_amd/build.py);
// the tag lets the build read it back from the .so without loading it
static const char kSourceHash[] = "surprise_amd-src-sha256:" MF_SOURCE_HASH;
const char *mf_source_hash(void) { return kSourceHash + 24; }

const char *mf_last_error(void) { return g_err; }

int mf_event_create(void **event)
{
    if (!event) return set_err(MF_E_ARG, "null event");
    hipEvent_t ev = nullptr;
    if (const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming); e != hipSuccess)
        return set_err((int)e, "hipEventCreateWithFlags failed");
    *event = (void *)ev;
    return 0;
}

int mf_event_destroy(void *event)
{
    if (!event) return 0;
    if (const hipError_t e = hipEventDestroy((hipEvent_t)event); e != hipSuccess)
        return set_err((int)e, "hipEventDestroy failed");
    return 0;
}

int mf_event_record(void *event, void *stream)
{
    if (!event) return set_err(MF_E_ARG, "null event");
    if (const hipError_t e = hipEventRecord((hipEvent_t)event, (hipStream_t)stream); e != hipSuccess)
        return set_err((int)e, "hipEventRecord failed");
    return 0;
}

int mf_stream_wait_event(void *stream, void *event)
{
    if (!event) return set_err(MF_E_ARG, "null event");
    if (const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0); e != hipSuccess)
        return set_err((int)e, "hipStreamWaitEvent failed");
    return 0;
}

int mf_launch_join(void *words, int32_t role, uint32_t epoch)
{
    if (words && role != 1 && role != 2) return set_err(MF_E_ARG, "join role must be 1 or 2");
    mf_ext::g_join = mf_ext::JoinArgs{(uint32_t *)words, words ? role : 0, epoch};
    return 0;
}

int mf_launch_fold(const mf_fold_t *f)
{
    mf_ext::g_fold = mf_ext::FoldArgs{};
    if (!f) return 0;
    if (!f->item_count || !f->words || !f->qb || !f->sums || !f->item_piece_ptr || !f->totals ||
        !f->hp)
        return set_err(MF_E_ARG, "mf_launch_fold: null argument");
    if (f->sums2 && !f->item_piece_ptr2) return set_err(MF_E_ARG, "sums2 needs item_piece_ptr2");
    if (f->role < 1 || f->role > 2 || f->n_launches < 1 || f->n_launches > 2 ||
        f->role > f->n_launches)
        return set_err(MF_E_ARG, "mf_launch_fold: role / n_launches");
    if (f->ld < 1 || f->n_factors < 0 || f->n_factors > f->ld || f->bias_col >= f->ld)
        return set_err(MF_E_ARG, "bad shape");
    if (f->rule != MF_MERGE_SUM && f->rule != MF_MERGE_COUNT && f->rule != MF_MERGE_RECENCY)
        return set_err(MF_E_ARG, "bad merge rule");
    const int count_rule = f->rule == MF_MERGE_COUNT ? 1 : (f->rule == MF_MERGE_RECENCY ? 2 : 0);
    if (count_rule && !f->p2stat) return set_err(MF_E_ARG, "count-aware rule needs p2stat");
    if (f->stat_next && f->stat_next == f->p2stat) return set_err(MF_E_ARG, "stat_next aliases p2stat");
    if (f->stat_next && (!f->user_sq || f->n_users < 0 || f->n_users >= kSqPartsMin))
        return set_err(MF_E_UNSUPPORTED, "mf_launch_fold: stat_next needs user_sq of < MF_SQ_PARTS_MIN users");
    if (f->bias_out && f->bias_col < 0) return set_err(MF_E_ARG, "bias_out needs bias_col");
    const mf_hyper_t *hp = f->hp;
    mf_ext::FoldArgs a;
    a.qb = f->qb;
    a.ipp_a = f->item_piece_ptr;
    a.ipp_b = f->sums2 ? f->item_piece_ptr2 : nullptr;
    a.sums_a = f->sums;
    a.sums_b = f->sums2;
    a.totals = f->totals;
    a.cnt = f->item_count;
    a.blk = f->words;
    a.p2stat = f->p2stat;
    a.stat_next = f->stat_next;
    a.user_sq = f->user_sq;
    a.bias_out = f->bias_out;
    a.n_users = f->n_users;
    a.ld = f->ld;
    a.n_fac = f->n_factors;
    a.bias_col = f->bias_col;
    a.count_rule = count_rule;
    a.role = f->role;
    a.n_launch = f->n_launches;
    // (mf_log_apply's constants)
    a.eta_b = count_rule ? hp->lr_bi * (1.0 + hp->reg_bi) : 0.0;
    a.lr_c = count_rule ? hp->lr_qi : 0.0;
    a.reg_c = count_rule ? hp->reg_qi : 0.0;
    a.lr_f = hp->lr_qi;
    a.reg_f = hp->reg_qi;
    a.lr_b = hp->lr_bi;
    a.reg_b = hp->reg_bi;
    mf_ext::g_fold = a;
    return 0;
}

int mf_launch_event(void *event)
{
    mf_ext::g_stop_event = (hipEvent_t)event;
    return 0;
}

int mf_svd_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                 int32_t ldu, void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                 const mf_hyper_t *hp, int32_t mode, void *qlog, void *elog, int32_t n_waves,
                 int32_t flags, int32_t dtype, void *stream)
{
    if (elog && mode != MF_MODE_LOG) return set_err(MF_E_ARG, "elog needs MF_MODE_LOG");
    return launch_epoch<false>(csr, sched, n_sched, pu, bu, ldu, qb, ldq, nullptr, qlog, elog,
                               n_factors, biased, hp, mode, n_waves, flags, dtype, stream);
}

int mf_svd_epoch_sq(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                    void *bu, int32_t ldu, void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                    const mf_hyper_t *hp, void *qlog, void *elog, double *user_sq,
                    const void *item_bias, int32_t n_waves, int32_t flags, int32_t dtype,
                    void *stream)
{
    if (!elog || !user_sq) return set_err(MF_E_ARG, "mf_svd_epoch_sq needs elog and user_sq");
    // (item_bias rides in the yj slot, which SVD does not use)
    return launch_epoch<false>(csr, sched, n_sched, pu, bu, ldu, qb, ldq,
                               const_cast<void *>(item_bias), qlog, elog, n_factors, biased, hp,
                               MF_MODE_LOG, n_waves, flags, dtype, stream, user_sq);
}

int mf_svd_epoch_gram(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                      void *bu, int32_t ldu, const void *qb, int32_t ldq, int32_t n_factors,
                      int32_t biased, const mf_hyper_t *hp, void *qlog, double *user_sq,
                      int32_t n_blocks, int32_t flags, int32_t dtype, void *stream)
{
    const int K = n_factors;
    if (int rc = check_epoch(csr, sched, pu, bu, qb, hp, K, ldu, ldq, MF_MODE_LOG, qlog, dtype))
        return rc;
    const int esz = dtype == MF_F32 ? 4 : 8;
    // (the row recursion runs one column per thread of three waves: ldq <= 192)
    if (K < 1 || (int64_t)ldq * esz > 1024 || ldq > 3 * kWave)
        return set_err(MF_E_UNSUPPORTED, "mf_svd_epoch_gram: 1 <= n_factors, rows of <= 1 KiB, "
                                         "ldq <= 192");
    const int err_col = err_column(K, ldq, dtype);
    if (err_col <= 0) return set_err(MF_E_UNSUPPORTED, "mf_svd_epoch_gram: no error columns");
    if (flags & ~(0xFF << MF_EPOCH_XCD_SHIFT))
        return set_err(MF_E_ARG, "mf_svd_epoch_gram: only the XCD mask flag");
    const int xmask = (flags >> MF_EPOCH_XCD_SHIFT) & 0xFF;
    if (int rc = check_xmask(xmask)) return rc;
    if (n_sched <= 0) return 0;
    int64_t blocks = n_blocks > 0 ? n_blocks : n_sched;
    if (xmask) {
        const int cnt = __builtin_popcount(xmask);
        blocks = 8 * ((blocks + cnt - 1) / cnt);
    }
    hipStream_t st = (hipStream_t)stream;
    const int ring = gram_ring_bytes(ldq, esz);
    if (dtype == MF_F32)
        hipLaunchKernelGGL(mf_svd_gram_kernel<float>, dim3((unsigned)blocks), dim3(kBlock), ring, st,
                           csr->row_ptr, csr->items, (const float *)csr->ratings, sched, n_sched,
                           (float *)pu, (float *)bu, ldu, (const float *)qb, ldq, K, biased,
                           cast_hyper<float>(hp), (float *)qlog, user_sq, err_col, xmask);
    else
        hipLaunchKernelGGL(mf_svd_gram_kernel<double>, dim3((unsigned)blocks), dim3(kBlock), ring, st,
                           csr->row_ptr, csr->items, (const double *)csr->ratings, sched, n_sched,
                           (double *)pu, (double *)bu, ldu, (const double *)qb, ldq, K, biased,
                           cast_hyper<double>(hp), (double *)qlog, user_sq, err_col, xmask);
    return check_launch("mf_svd_gram_kernel");
}

int mf_svdpp_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                   int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                   const mf_hyper_t *hp, int32_t mode, void *qlog, void *ycbuf, int32_t n_waves,
                   int32_t flags, int32_t *status, const uint8_t *hot, int32_t dtype, void *stream)
{
    return launch_epoch<true>(csr, sched, n_sched, pu, bu, ldu, qb, ldq, yj, qlog, ycbuf,
                              n_factors, 1, hp, mode, n_waves, flags, dtype, stream, nullptr,
                              status, hot);
}

int mf_svdpp_epoch_qlog(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                        void *bu, int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                        const mf_hyper_t *hp, void *qlog, const int64_t *log_row0, void *ycbuf,
                        double *user_sq, int32_t n_waves, int32_t flags, int32_t dtype,
                        void *stream)
{
    if (!qlog || !log_row0 || !ycbuf) return set_err(MF_E_ARG, "the q log needs qlog, log_row0, ycbuf");
    if (flags & ~(MF_EPOCH_DUP_ITEMS | MF_EPOCH_LOG_NT | (0xFF << MF_EPOCH_XCD_SHIFT)))
        return set_err(MF_E_ARG, "mf_svdpp_epoch_qlog: flags MF_EPOCH_DUP_ITEMS / MF_EPOCH_LOG_NT / "
                                 "XCD mask only");
    return launch_epoch<true>(csr, sched, n_sched, pu, bu, ldu, qb, ldq, yj, qlog, ycbuf,
                              n_factors, 1, hp, MF_MODE_LOG, n_waves, flags, dtype, stream,
                              user_sq, nullptr, nullptr, log_row0);
}

int mf_svdpp_epoch_mix(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                       void *bu, int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                       const mf_hyper_t *hp, void *cold_log, const int32_t *cold_row,
                       void *ycbuf, double *user_sq, int32_t n_waves, int32_t flags,
                       int32_t *status, const uint8_t *hot, int32_t dtype, void *stream)
{
    if (!cold_log || !cold_row || !ycbuf || !user_sq)
        return set_err(MF_E_ARG, "the hybrid launch needs cold_log, cold_row, ycbuf and user_sq");
    if (!(flags & MF_EPOCH_SVDPP_HELPERS) || (flags & MF_EPOCH_SVDPP_ONE_HELPER))
        return set_err(MF_E_ARG, "the hybrid launch: MF_EPOCH_SVDPP_HELPERS (three helpers)");
    // ring slots carry byte offsets with bit 31 marking a cold-log row (kColdSlot): every q
    // offset, hot-row replicas included, must stay below 2 GiB
    const uint64_t esz = dtype == MF_F32 ? 4 : 8;
    if (csr && (uint64_t)csr->n_items * (hot ? 2 : 1) * (uint64_t)(ldq > 0 ? ldq : 0) * esz >=
                   kMaxTable)
        return set_err(MF_E_UNSUPPORTED, "the hybrid launch: item table (with replicas) >= 2 GiB");
    return launch_epoch<true>(csr, sched, n_sched, pu, bu, ldu, qb, ldq, yj, cold_log, ycbuf,
                              n_factors, 1, hp, MF_MODE_ATOMIC, n_waves, flags, dtype, stream,
                              user_sq, status, hot, nullptr, cold_row);
}

int mf_svdpp_hot_fold(void *qb, int32_t ldq, int32_t n_items, const int32_t *hot_items,
                      int32_t n_hot, int32_t dtype, void *stream)
{
    if (n_hot < 0 || n_items < 0 || ldq <= 0) return set_err(MF_E_ARG, "bad argument");
    if (n_hot == 0) return 0;
    if (!qb || !hot_items) return set_err(MF_E_ARG, "null pointer");
    const int64_t total = (int64_t)n_hot * ldq;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(hot_fold_kernel<float>, dim3(elementwise_grid(total)), dim3(kBlock), 0,
                           st, (float *)qb, ldq, n_items, hot_items, total);
    else
        hipLaunchKernelGGL(hot_fold_kernel<double>, dim3(elementwise_grid(total)), dim3(kBlock), 0,
                           st, (double *)qb, ldq, n_items, hot_items, total);
    return check_launch("hot_fold_kernel");
}

int mf_sumsq(const void *x, int64_t n_rows, int32_t n_cols, int32_t ld, double *out, int32_t dtype,
             void *stream)
{
    if (!out || n_rows < 0 || n_cols < 0 || ld < n_cols) return set_err(MF_E_ARG, "bad argument");
    if (n_rows == 0 || n_cols == 0) return 0;
    if (!x) return set_err(MF_E_ARG, "null x");
    // <= 256 blocks (one double atomic each: more contend on the two words, measured 14 us at
    // 1500 blocks vs 7 at 256 on ML-1M), rows unrolled by 4 inside the kernel
    const int g = grid_for_waves(n_rows < 1024 ? n_rows : 1024);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(sumsq_kernel<float>, dim3(g), dim3(kBlock), 0, st, (const float *)x,
                           n_rows, n_cols, ld, out);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(sumsq_kernel<double>, dim3(g), dim3(kBlock), 0, st, (const double *)x,
                           n_rows, n_cols, ld, out);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("sumsq_kernel");
}

int mf_user_sq(const void *pu, int64_t n_rows, int32_t n_cols, int32_t ld, double *user_sq,
               int32_t dtype, void *stream)
{
    if (!user_sq || n_rows < 0 || n_cols < 0 || ld < n_cols) return set_err(MF_E_ARG, "bad argument");
    if (n_rows == 0) return 0;
    if (!pu) return set_err(MF_E_ARG, "null pu");
    const int g = grid_for_waves(n_rows < 4096 ? n_rows : 4096);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(user_sq_kernel<float>, dim3(g), dim3(kBlock), 0, st, (const float *)pu,
                           n_rows, n_cols, ld, user_sq);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(user_sq_kernel<double>, dim3(g), dim3(kBlock), 0, st, (const double *)pu,
                           n_rows, n_cols, ld, user_sq);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("user_sq_kernel");
}

int mf_user_sq_reduce(const double *user_sq, int64_t n_rows, int32_t n_cols, double *out,
                      void *stream)
{
    if (!out || n_rows < 0 || n_cols < 0 || (n_rows > 0 && !user_sq))
        return set_err(MF_E_ARG, "bad argument");
    if (int e = launch_sq_parts(user_sq, n_rows, out, (hipStream_t)stream)) return e;
    hipLaunchKernelGGL(user_sq_reduce_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream,
                       user_sq, n_rows, n_cols, out);
    return check_launch("user_sq_reduce_kernel");
}

int mf_log_reduce(const void *qlog, int32_t ld, int32_t n_cols, const int32_t *perm,
                  const int32_t *piece_beg, int64_t n_pieces, void *sums,
                  const int32_t *piece_item, const mf_hyper_t *hp, const mf_recency_t *rec,
                  int32_t dtype, void *stream)
{
    if (n_pieces < 0 || ld < 1 || n_cols < 1 || n_cols > ld) return set_err(MF_E_ARG, "bad shape");
    if (n_pieces == 0) return 0;
    if (!qlog || !perm || !piece_beg || !sums) return set_err(MF_E_ARG, "null argument");
    Recency rc;
    if (int e = make_recency(rec, hp, rc)) return e;
    if (rec && !piece_item) return set_err(MF_E_ARG, "recency weights need piece_item");
    const int g = grid_for_waves(default_waves(n_pieces));
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_g<T>(ld, [&](auto gc) -> int {
            constexpr int V = decltype(gc)::value;
            if (rec)
                hipLaunchKernelGGL((log_reduce_kernel<T, V, true>), dim3(g), dim3(kBlock), 0, st,
                                   (const T *)qlog, ld, n_cols, perm, piece_beg, n_pieces,
                                   (T *)sums, (const int32_t *)nullptr, piece_item, rc, n_cols - 1);
            else
                hipLaunchKernelGGL((log_reduce_kernel<T, V, false>), dim3(g), dim3(kBlock), 0, st,
                                   (const T *)qlog, ld, n_cols, perm, piece_beg, n_pieces,
                                   (T *)sums, (const int32_t *)nullptr, piece_item, rc, n_cols - 1);
            return check_launch("log_reduce_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_log_replay(const void *qlog, const void *elog, int32_t ldq, int32_t n_factors,
                  const mf_csr_t *csr, const void *qb, const mf_hyper_t *hp, const int32_t *perm,
                  const int32_t *ck_pos, const int32_t *piece_beg, int64_t n_pieces, void *sums,
                  const int32_t *piece_item, const mf_recency_t *rec, int32_t flags,
                  int32_t dtype, void *stream)
{
    StopEvent stop(stream);  // (mf_launch_event)
    const mf_ext::JoinArgs join = mf_ext::take_join();  // (mf_launch_join)
    const mf_ext::FoldArgs fold = mf_ext::take_fold();  // (mf_launch_fold)
    if (n_pieces < 0 || ldq < n_factors + 1 || n_factors < 0) return set_err(MF_E_ARG, "bad shape");
    if (fold.cnt && join.words) return set_err(MF_E_ARG, "mf_launch_fold with mf_launch_join");
    if (fold.cnt && fold.ld != ldq) return set_err(MF_E_ARG, "mf_launch_fold: ld != ldq");
    if (fold.cnt && !rec) return set_err(MF_E_UNSUPPORTED, "mf_launch_fold: recency weights only");
    const int xmask = (flags >> MF_EPOCH_XCD_SHIFT) & 0xFF;
    if (int rc = check_xmask(xmask)) return rc;
    // (a join or a fold still launches: its partner waits / its blocks count for the statistic)
    if (n_pieces == 0 && !join.words && !fold.cnt) return 0;
    if (!qlog || !elog || !csr || !qb || !hp || !perm || !ck_pos || !piece_beg || !sums)
        return set_err(MF_E_ARG, "null argument");
    const int err_col = (flags & MF_EPOCH_ERR_IN_ROW) ? err_column(n_factors, ldq, dtype) : 0;
    if ((flags & MF_EPOCH_ERR_IN_ROW) && err_col <= 0)
        return set_err(MF_E_UNSUPPORTED, "MF_EPOCH_ERR_IN_ROW: no spare columns");
    if ((flags & MF_EPOCH_CKPT_NARROW) && (err_col || n_factors < 1))
        return set_err(MF_E_ARG, "MF_EPOCH_CKPT_NARROW: errors in elog, n_factors >= 1");
    const int ldc = (flags & MF_EPOCH_CKPT_NARROW) ? ckpt_narrow_ld(n_factors, dtype) : ldq;
    const int64_t esz = dtype == MF_F64 ? 8 : 4;
    // rows of <= 1 KiB; narrow rows: their factor columns in <= 1 KiB, the item row / sums in one
    // more lane group at most (fp64 K = 128: ldc 128, ldq 136)
    if ((int64_t)ldc * esz > 512 * kLaMaxG || (ldc == ldq && (int64_t)ldq * esz > 512 * kLaMaxG) ||
        (int64_t)ldq * esz > 512 * (kLaMaxG + 1))
        return set_err(MF_E_UNSUPPORTED, "checkpoint log: ldq * size <= 1 KiB (narrow rows: ldc) only");
    Recency rc;
    if (int e = make_recency(rec, hp, rc)) return e;
    const int wpc = (flags >> MF_REPLAY_WPC_SHIFT) & 0xFF;
    const int64_t cap = (int64_t)n_cus() * (wpc ? wpc : MF_REPLAY_WPC) *
                        (xmask ? __builtin_popcount(xmask) : 8) / 8;
    const int g = grid_for_waves_x(n_pieces < 1 ? 1 : n_pieces < cap ? n_pieces : cap, xmask);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_g<T>(ldq, [&](auto gc) -> int {
            constexpr int V = decltype(gc)::value;
            if constexpr (V > kLaMaxG + 1) {
                return set_err(MF_E_UNSUPPORTED, "checkpoint log: row too long");
            } else {
                // (V = kLaMaxG + 1 only for narrow rows: their groups stop at kLaMaxG)
                // (the fold inside the replay: recency rule only -- the default)
                auto kern = fold.cnt ? log_replay_kernel<T, V, true, true>
                            : rec    ? log_replay_kernel<T, V, true, false>
                                     : log_replay_kernel<T, V, false, false>;
                launch_ev(stop.take(), kern, dim3(g), dim3(kBlock), st,
                                   (const T *)qlog, (const T *)elog, ldq, n_factors, csr->items,
                                   (const T *)qb, csr->n_items, (T)hp->lr_pu,
                                   (T)(1.0 / (1.0 - hp->lr_pu * hp->reg_pu)), perm,
                                   ck_pos, piece_beg, n_pieces, (T *)sums, xmask, err_col,
                                   piece_item, join.words, join.role, join.epoch, rc, ldc, fold);
                return check_launch("log_replay_kernel");
            }
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_ckpt_interval(void) { return kCkpt; }

int mf_svdpp_y_fold(void *yj, int32_t ldu, int32_t n_factors, const void *ycbuf, const void *uA,
                    const int32_t *item_users, const int32_t *piece_beg, int64_t n_pieces,
                    const int32_t *item_piece_ptr, int32_t n_items, void *piece_c,
                    void *piece_A, const int32_t *piece_item, int32_t dtype, void *stream)
{
    if (n_items < 0 || n_pieces < 0 || ldu < n_factors || n_factors < 0)
        return set_err(MF_E_ARG, "bad shape");
    if (n_items == 0 || n_pieces == 0 || n_factors == 0) return 0;
    if (!yj || !ycbuf || !uA || !item_users || !piece_beg || !item_piece_ptr || !piece_c ||
        !piece_A)
        return set_err(MF_E_ARG, "null argument");
    const int gp = grid_for_waves(default_waves(n_pieces));
    const int gi = grid_for_waves(default_waves(n_items));
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T>(ldu, [&](auto vc) -> int {
            constexpr int V = decltype(vc)::value;
            hipLaunchKernelGGL((y_piece_kernel<T, V>), dim3(gp), dim3(kBlock), 0, st, ldu,
                               n_factors, (const T *)ycbuf, (const T *)uA, item_users, piece_beg,
                               n_pieces, (T *)piece_c, (T *)piece_A, piece_item, item_piece_ptr,
                               (T *)yj);
            if (int rc = check_launch("y_piece_kernel")) return rc;
            hipLaunchKernelGGL((y_apply_kernel<T, V>), dim3(gi), dim3(kBlock), 0, st, (T *)yj,
                               ldu, n_factors, item_piece_ptr, n_items, (const T *)piece_c,
                               (const T *)piece_A, piece_item ? 2 : 1);
            return check_launch("y_apply_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_svdpp_qlog_fold(void *qb, int32_t ldq, int32_t n_factors, void *yj, int32_t ldu,
                       const void *qlog, const mf_qlog_fold_t *lay, const int32_t *totals,
                       const double *p2stat, const mf_hyper_t *hp, const void *ycbuf,
                       const void *uA, int32_t n_items, double *stat_next,
                       const double *user_sq, int64_t n_users, int32_t dtype, void *stream)
{
    if (n_items < 0 || n_factors < 1 || ldq < n_factors + 1 || ldu < n_factors)
        return set_err(MF_E_ARG, "bad shape");
    if (!qb || !yj || !qlog || !lay || !totals || !p2stat || !hp || !ycbuf || !uA ||
        !lay->perm || !lay->rpos || !lay->item_row_beg || !lay->users)
        return set_err(MF_E_ARG, "null argument");
    const bool hot = lay->n_hot_pieces > 0;
    if (hot && (!lay->hot_perm || !lay->hot_rpos || !lay->hot_users || !lay->hot_piece_beg ||
                !lay->hot_piece_item || !lay->hot_item_piece_ptr || !lay->hot_sums ||
                !lay->hot_piece_c || !lay->hot_piece_A))
        return set_err(MF_E_ARG, "null hot-item argument");
    if (user_sq && (!stat_next || n_users < 0)) return set_err(MF_E_ARG, "user_sq needs stat_next");
    if (stat_next && stat_next == p2stat) return set_err(MF_E_ARG, "stat_next aliases p2stat");
    if (n_items == 0) return 0;
    mf_recency_t cold_rec{lay->rpos, nullptr, totals, p2stat};
    mf_recency_t hot_rec{lay->hot_rpos, nullptr, totals, p2stat};
    Recency rc, rch;
    if (int e = make_recency(&cold_rec, hp, rc)) return e;
    if (hot) {
        if (int e = make_recency(&hot_rec, hp, rch)) return e;
    }
    // (waves take batches of 64 items)
    const int64_t nb = ((int64_t)n_items + kWave - 1) / kWave, cap = (int64_t)n_cus() * kFoldWPC;
    const int g = grid_for_waves(nb < cap ? nb : cap) + (stat_next ? 1 : 0);
    const int gh = hot ? grid_for_waves(default_waves(lay->n_hot_pieces)) : 0;
    hipStream_t st = (hipStream_t)stream;
    if (int e = launch_sq_parts(user_sq, n_users, stat_next, st)) return e;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        // the hot items' pre-passes: piece sums of their gradient rows (log_reduce_kernel) and
        // piece maps of their users' y updates (y_piece_kernel)
        if (hot) {
            int rc_g = dispatch_g<T>(ldq, [&](auto gc) -> int {
                constexpr int V = decltype(gc)::value;
                hipLaunchKernelGGL((log_reduce_kernel<T, V, true>), dim3(gh), dim3(kBlock), 0, st,
                                   (const T *)qlog, ldq, n_factors + 1, lay->hot_perm,
                                   lay->hot_piece_beg, lay->n_hot_pieces, (T *)lay->hot_sums,
                                   (const int32_t *)nullptr, lay->hot_piece_item, rch, n_factors);
                return check_launch("log_reduce_kernel");
            });
            if (rc_g) return rc_g;
            int rc_y = dispatch_v<T>(ldu, [&](auto vc) -> int {
                constexpr int V = decltype(vc)::value;
                hipLaunchKernelGGL((y_piece_kernel<T, V>), dim3(gh), dim3(kBlock), 0, st, ldu,
                                   n_factors, (const T *)ycbuf, (const T *)uA, lay->hot_users,
                                   lay->hot_piece_beg, lay->n_hot_pieces, (T *)lay->hot_piece_c,
                                   (T *)lay->hot_piece_A, (const int32_t *)nullptr,
                                   (const int32_t *)nullptr, (T *)yj);
                return check_launch("y_piece_kernel");
            });
            if (rc_y) return rc_y;
        }
        return dispatch_v<T>(ldq, [&](auto vq) -> int {
            constexpr int VQ = decltype(vq)::value;
            return dispatch_v<T>(ldu, [&](auto vy) -> int {
                constexpr int VY = decltype(vy)::value;
                if constexpr (VQ > 5 || VY > VQ || VQ - VY > 1) {
                    return set_err(MF_E_UNSUPPORTED, "the fused fold: rows of <= 320 columns");
                } else {
                    hipLaunchKernelGGL((qlog_fold_kernel<T, VQ, VY>), dim3(g), dim3(kBlock), 0, st,
                                       (T *)qb, ldq, n_factors, (T *)yj, ldu, (const T *)qlog,
                                       lay->perm, lay->item_row_beg, totals, rc, hp->lr_qi,
                                       hp->reg_qi, hp->lr_bi, hp->reg_bi, (const T *)ycbuf,
                                       (const T *)uA, lay->users, n_items,
                                       stat_next, user_sq, n_users, n_factors,
                                       (const T *)(hot ? lay->hot_sums : nullptr),
                                       hot ? lay->hot_item_piece_ptr : nullptr,
                                       (const T *)(hot ? lay->hot_piece_c : nullptr),
                                       (const T *)(hot ? lay->hot_piece_A : nullptr));
                    return check_launch("qlog_fold_kernel");
                }
            });
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_log_apply(void *qb, int32_t n_items, int32_t ld, int32_t n_factors, int32_t bias_col,
                 const void *sums, const int32_t *item_piece_ptr, const void *sums2,
                 const int32_t *item_piece_ptr2, const int32_t *totals, const mf_hyper_t *hp,
                 const double *p2stat, int32_t rule, void *delta_out, int32_t apply,
                 double *stat_next, const double *user_sq, int64_t n_users, void *bias_out,
                 int32_t dtype, void *stream)
{
    if (bias_out && (!apply || bias_col < 0)) return set_err(MF_E_ARG, "bias_out needs apply and bias_col");
    StopEvent stop(stream);  // (mf_launch_event)
    if (stat_next && stat_next == p2stat) return set_err(MF_E_ARG, "stat_next aliases p2stat");
    if (user_sq && (!stat_next || n_users < 0)) return set_err(MF_E_ARG, "user_sq needs stat_next");
    if (sums2 && !item_piece_ptr2) return set_err(MF_E_ARG, "sums2 needs item_piece_ptr2");
    if (n_items < 0 || ld < 1 || n_factors < 0 || n_factors > ld || bias_col >= ld)
        return set_err(MF_E_ARG, "bad shape");
    if (rule != MF_MERGE_SUM && rule != MF_MERGE_COUNT && rule != MF_MERGE_RECENCY)
        return set_err(MF_E_ARG, "bad merge rule");
    // (0 plain sum, 1 count-aware weight, 2 recency: sums weighted by the replay / reduce)
    const int count_rule = rule == MF_MERGE_COUNT ? 1 : (rule == MF_MERGE_RECENCY ? 2 : 0);
    if (count_rule && (!totals || !hp || !p2stat))
        return set_err(MF_E_ARG, "count-aware rule needs totals, hp, p2stat");
    if (apply && (!totals || !hp)) return set_err(MF_E_ARG, "apply needs totals and hp");
    if (n_items == 0 || (!apply && !delta_out)) return 0;
    if (!sums || (apply && !qb)) return set_err(MF_E_ARG, "null argument");
    // (+1: the block that sums / clears stat_next)
    const int g = grid_for_waves(default_waves(n_items)) + (stat_next ? 1 : 0);
    hipStream_t st = (hipStream_t)stream;
    if (int e = launch_sq_parts(user_sq, n_users, stat_next, st)) return e;
    const double eta_b = count_rule ? hp->lr_bi * (1.0 + hp->reg_bi) : 0.0;
    const double lr_c = count_rule ? hp->lr_qi : 0.0, reg_c = count_rule ? hp->reg_qi : 0.0;
    const double lr_f = hp ? hp->lr_qi : 0.0, reg_f = hp ? hp->reg_qi : 0.0;
    const double lr_b = hp ? hp->lr_bi : 0.0, reg_b = hp ? hp->reg_bi : 0.0;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T>(ld, [&](auto vc) -> int {
            if (sums2)
                launch_ev(stop.take(), (log_apply_kernel<T, decltype(vc)::value, true>), dim3(g), dim3(kBlock),
                               st, (T *)qb, n_items, ld, n_factors, bias_col, (const T *)sums,
                               item_piece_ptr, (const T *)sums2, item_piece_ptr2, totals,
                               count_rule, eta_b, lr_c, reg_c, lr_f,
                               reg_f, lr_b, reg_b, p2stat, (T *)delta_out, apply, stat_next,
                               user_sq, (int64_t)n_users, n_factors, (T *)bias_out);
            else
                launch_ev(stop.take(), (log_apply_kernel<T, decltype(vc)::value, false>), dim3(g), dim3(kBlock),
                               st, (T *)qb, n_items, ld, n_factors, bias_col, (const T *)sums,
                               item_piece_ptr, (const T *)sums2, item_piece_ptr2, totals,
                               count_rule, eta_b, lr_c, reg_c, lr_f,
                               reg_f, lr_b, reg_b, p2stat, (T *)delta_out, apply, stat_next,
                               user_sq, (int64_t)n_users, n_factors, (T *)bias_out);
            return check_launch("log_apply_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_item_merge(void *tab, void *snap, int32_t n_items, int32_t ld, int32_t n_factors,
                  int32_t bias_col, int32_t n_replicas, int32_t rule, const int32_t *counts,
                  const int32_t *totals, const mf_hyper_t *hp, const void *pu, int32_t n_users,
                  int32_t ldu, void *work, void *delta_out, int32_t apply, int32_t dtype,
                  void *stream)
{
    if (!tab || !snap || n_items < 0 || ld < 1 || n_replicas < 1)
        return set_err(MF_E_ARG, "bad item table");
    if (rule < MF_MERGE_SUM || rule > MF_MERGE_RECENCY) return set_err(MF_E_ARG, "bad merge rule");
    if (rule == MF_MERGE_SUM) counts = nullptr;
    const int mean = rule == MF_MERGE_MEAN;
    if (counts && !totals && rule != MF_MERGE_RECENCY)
        return set_err(MF_E_ARG, "counted merge needs totals");
    if (counts && !mean && (!hp || !pu || !work || n_users < 1 || ldu < n_factors))
        return set_err(MF_E_ARG, "count-aware merge needs hp, pu, work");
    if (rule != MF_MERGE_SUM && !counts) return set_err(MF_E_ARG, "counted merge needs counts");
    if (dtype != MF_F32 && dtype != MF_F64) return set_err(MF_E_ARG, "bad dtype");
    if (!delta_out && !apply) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int64_t total = (int64_t)n_items * ld;
    double l1m_bias = 0, lr_fac = 0, reg_fac = 0;
    if (counts && !mean) {
        l1m_bias = bias_col >= 0 ? log1p(-hp->lr_bi * (1.0 + hp->reg_bi)) : 0.0;
        lr_fac = hp->lr_qi;
        reg_fac = hp->reg_qi;
        hipError_t e = hipMemsetAsync(work, 0, 2 * sizeof(double), st);
        if (e != hipSuccess) return set_err((int)e, "hipMemsetAsync(work)");
        const int g = grid_for_waves(n_users < 1024 ? n_users : 1024);
        if (dtype == MF_F32)
            hipLaunchKernelGGL(sumsq_kernel<float>, dim3(g), dim3(kBlock), 0, st, (const float *)pu,
                               (int64_t)n_users, n_factors, ldu, (double *)work);
        else
            hipLaunchKernelGGL(sumsq_kernel<double>, dim3(g), dim3(kBlock), 0, st,
                               (const double *)pu, (int64_t)n_users, n_factors, ldu, (double *)work);
        if (int rc = check_launch("sumsq_kernel")) return rc;
    }
    const int g = elementwise_grid(total);
    if (dtype == MF_F32)
        hipLaunchKernelGGL(item_merge_kernel<float>, dim3(g), dim3(kBlock), 0, st, (float *)tab,
                           (float *)snap, n_items, ld, n_factors, bias_col, n_replicas, counts,
                           totals, rule, l1m_bias, lr_fac, reg_fac, (const double *)work,
                           (float *)delta_out, apply);
    else
        hipLaunchKernelGGL(item_merge_kernel<double>, dim3(g), dim3(kBlock), 0, st, (double *)tab,
                           (double *)snap, n_items, ld, n_factors, bias_col, n_replicas, counts,
                           totals, rule, l1m_bias, lr_fac, reg_fac, (const double *)work,
                           (double *)delta_out, apply);
    return check_launch("item_merge_kernel");
}

int mf_item_apply(void *tab, void *snap, int32_t n_items, int32_t ld, int32_t n_replicas,
                  const void *delta, int32_t dtype, void *stream)
{
    if (!tab || !snap || !delta || n_replicas < 1) return set_err(MF_E_ARG, "bad argument");
    const int64_t total = (int64_t)n_items * ld;
    const int g = elementwise_grid(total);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(item_apply_kernel<float>, dim3(g), dim3(kBlock), 0, st, (float *)tab,
                           (float *)snap, total, n_replicas, (const float *)delta);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(item_apply_kernel<double>, dim3(g), dim3(kBlock), 0, st, (double *)tab,
                           (double *)snap, total, n_replicas, (const double *)delta);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("item_apply_kernel");
}

int mf_item_affine(void *tab, void *snap, int32_t n_items, int32_t ld, const void *a,
                   const void *s, void *delta, int32_t phase, int32_t dtype, void *stream)
{
    if (!tab || !snap || !a || !delta || n_items < 0 || ld < 1 || (phase != 0 && phase != 1) ||
        (phase == 0 && !s))
        return set_err(MF_E_ARG, "bad argument");
    if (n_items == 0) return 0;
    const int g = elementwise_grid((int64_t)n_items * ld);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(item_affine_kernel<float>, dim3(g), dim3(kBlock), 0, st, (float *)tab,
                           (float *)snap, n_items, ld, (const float *)a, (const float *)s,
                           (float *)delta, phase);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(item_affine_kernel<double>, dim3(g), dim3(kBlock), 0, st, (double *)tab,
                           (double *)snap, n_items, ld, (const double *)a, (const double *)s,
                           (double *)delta, phase);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("item_affine_kernel");
}

int mf_nmf_user_pass(const mf_csr_t *csr, const void *pu, void *pu_next, void *bu, int32_t ldu,
                     const void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                     const mf_hyper_t *hp, void *est, void *blog, const int64_t *piece_beg,
                     int64_t n_pieces, const int32_t *user_piece_ptr, const int32_t *piece_user,
                     void *scratch, int32_t dtype, void *stream)
{
    if (!csr || !csr->row_ptr || !csr->items || !csr->ratings) return set_err(MF_E_ARG, "null csr");
    if (!pu || !pu_next || !qb || !hp || !est || (biased && (!bu || !blog)))
        return set_err(MF_E_ARG, "null argument");
    if (n_factors < 1 || ldu < n_factors || ldq < n_factors + 1)
        return set_err(MF_E_ARG, "need ldu >= n_factors >= 1, ldq >= n_factors+1");
    if (csr->n_users <= 0) return 0;
    const int g = grid_for_waves(default_waves(csr->n_users));
    hipStream_t st = (hipStream_t)stream;
    const int width = ldu > ldq ? ldu : ldq;
    const bool pieces = piece_beg && user_piece_ptr && piece_user && scratch && n_pieces > 0;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        if (!biased) {
            const int rc = dispatch_seg<T>(width, [&](auto sc, auto ec) -> int {
                constexpr int S = decltype(sc)::value, E = decltype(ec)::value;
                if (pieces) {
                    hipLaunchKernelGGL((nmf_user_piece_kernel<T, S, E>),
                                       dim3(grid_for_waves(default_waves(n_pieces))), dim3(kBlock),
                                       0, st, csr->items, (const T *)csr->ratings, (const T *)pu,
                                       ldu, (const T *)qb, ldq, n_factors, piece_beg, piece_user,
                                       n_pieces, (T *)scratch, (T *)est);
                    if (int e = check_launch("nmf_user_piece_kernel")) return e;
                    hipLaunchKernelGGL(nmf_user_fold_kernel<T>, dim3(g), dim3(kBlock), 0, st,
                                       csr->row_ptr, user_piece_ptr, csr->n_users,
                                       (const T *)scratch, (const T *)pu, (T *)pu_next, ldu,
                                       n_factors, (T)hp->reg_pu);
                    return check_launch("nmf_user_fold_kernel");
                }
                hipLaunchKernelGGL((nmf_user_seg_kernel<T, S, E>), dim3(g), dim3(kBlock), 0, st,
                                   csr->row_ptr, csr->items, (const T *)csr->ratings,
                                   csr->n_users, (const T *)pu, (T *)pu_next, ldu, (const T *)qb,
                                   ldq, n_factors, (T)hp->reg_pu, (T *)est);
                return check_launch("nmf_user_seg_kernel");
            });
            if (rc >= 0) return rc;
        }
        return dispatch_g<T>(ldq, [&](auto gc) -> int {
            constexpr int G = decltype(gc)::value;
            auto k = biased ? nmf_user_kernel<T, G, true> : nmf_user_kernel<T, G, false>;
            hipLaunchKernelGGL(k, dim3(g), dim3(kBlock), 0, st, csr->row_ptr, csr->items,
                               (const T *)csr->ratings, csr->n_users, (const T *)pu, (T *)pu_next,
                               (T *)bu, ldu, (const T *)qb, ldq, n_factors, (T)hp->reg_pu,
                               (T)hp->lr_bu, (T)hp->reg_bu, (T)hp->lr_bi, (T)hp->reg_bi,
                               (T)hp->global_mean, (T *)est, (T *)blog);
            return check_launch("nmf_user_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_nmf_item_pass(const int64_t *csc_ptr, const int64_t *csc_pos, const int32_t *row_user,
                     const void *ratings, const void *est, const void *blog, const void *pu,
                     int32_t ldu, void *qb, int32_t ldq, int32_t n_items, int32_t n_factors,
                     int32_t biased, const mf_hyper_t *hp, int32_t rule,
                     const int64_t *piece_beg, int64_t n_pieces, const int32_t *item_piece_ptr,
                     void *scratch, const void *csc_ratings, const int32_t *csc_user,
                     int32_t dtype, void *stream)
{
    if (!csc_ptr || !csc_pos || !row_user || !ratings || !est || !pu || !qb || !hp ||
        (biased && !blog))
        return set_err(MF_E_ARG, "null argument");
    if (n_factors < 1 || ldu < n_factors || ldq < n_factors + 1)
        return set_err(MF_E_ARG, "need ldu >= n_factors >= 1, ldq >= n_factors+1");
    if (rule != MF_MERGE_SUM && rule != MF_MERGE_COUNT) return set_err(MF_E_ARG, "bad merge rule");
    if (n_items <= 0) return 0;
    const int g = grid_for_waves(default_waves(n_items));
    hipStream_t st = (hipStream_t)stream;
    const double eta_b = hp->lr_bi * (1.0 + hp->reg_bi);
    const int width = ldu > ldq ? ldu : ldq;
    const bool pieces = piece_beg && item_piece_ptr && scratch && n_pieces > 0;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        const int rc = dispatch_seg<T>(width, [&](auto sc, auto ec) -> int {
            constexpr int S = decltype(sc)::value, E = decltype(ec)::value;
            if (pieces) {
                auto kp = biased ? nmf_item_piece_kernel<T, S, E, true>
                                 : nmf_item_piece_kernel<T, S, E, false>;
                hipLaunchKernelGGL(kp, dim3(grid_for_waves(default_waves(n_pieces))), dim3(kBlock),
                                   0, st, csc_pos, row_user, (const T *)ratings, (const T *)est,
                                   (const T *)blog, (const T *)pu, ldu, ldq, piece_beg, n_pieces,
                                   (T *)scratch, (const T *)csc_ratings, csc_user);
                if (int e = check_launch("nmf_item_piece_kernel")) return e;
                hipLaunchKernelGGL(nmf_item_fold_kernel<T>, dim3(g), dim3(kBlock), 0, st, csc_ptr,
                                   item_piece_ptr, n_items, (const T *)scratch, (T *)qb, ldq,
                                   n_factors, (T)hp->reg_qi, biased, eta_b,
                                   rule == MF_MERGE_COUNT);
                return check_launch("nmf_item_fold_kernel");
            }
            auto k = biased ? nmf_item_seg_kernel<T, S, E, true> : nmf_item_seg_kernel<T, S, E, false>;
            hipLaunchKernelGGL(k, dim3(g), dim3(kBlock), 0, st, csc_ptr, csc_pos, row_user,
                               (const T *)ratings, (const T *)est, (const T *)blog, (const T *)pu,
                               ldu, (T *)qb, ldq, n_factors, n_items, (T)hp->reg_qi, eta_b,
                               rule == MF_MERGE_COUNT);
            return check_launch("nmf_item_seg_kernel");
        });
        if (rc >= 0) return rc;
        return dispatch_g<T>(ldq, [&](auto gc) -> int {
            constexpr int G = decltype(gc)::value;
            auto k = biased ? nmf_item_kernel<T, G, true> : nmf_item_kernel<T, G, false>;
            hipLaunchKernelGGL(k, dim3(g), dim3(kBlock), 0, st, csc_ptr, csc_pos, row_user,
                               (const T *)ratings, (const T *)est, (const T *)blog, (const T *)pu,
                               ldu, (T *)qb, ldq, n_factors, n_items, (T)hp->reg_qi, eta_b,
                               rule == MF_MERGE_COUNT);
            return check_launch("nmf_item_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_baseline_als_epoch(const mf_csr_t *csr, const int64_t *csc_ptr, const int64_t *csc_pos,
                          const int32_t *row_user, void *bu, void *bi, double global_mean,
                          double reg_u, double reg_i, const void *csc_ratings,
                          const int32_t *csc_user, int32_t dtype, void *stream)
{
    if (!csr || !csr->row_ptr || !csr->items || !csr->ratings) return set_err(MF_E_ARG, "null csr");
    if (!csc_ptr || !csc_pos || !row_user || !bu || !bi) return set_err(MF_E_ARG, "null argument");
    hipStream_t st = (hipStream_t)stream;
    const int gi = grid_for_waves(default_waves(csr->n_items > 0 ? csr->n_items : 1));
    const int gu = grid_for_waves(default_waves(csr->n_users > 0 ? csr->n_users : 1));
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        if (csr->n_items > 0) {
            hipLaunchKernelGGL(als_item_kernel<T>, dim3(gi), dim3(kBlock), 0, st, csc_ptr, csc_pos,
                               row_user, (const T *)csr->ratings, (const T *)bu, (T *)bi,
                               csr->n_items, (T)global_mean, (T)reg_i, (const T *)csc_ratings,
                               csc_user);
            if (int rc = check_launch("als_item_kernel")) return rc;
        }
        if (csr->n_users > 0) {
            hipLaunchKernelGGL(als_user_kernel<T>, dim3(gu), dim3(kBlock), 0, st, csr->row_ptr,
                               csr->items, (const T *)csr->ratings, (const T *)bi, (T *)bu,
                               csr->n_users, (T)global_mean, (T)reg_u);
            if (int rc = check_launch("als_user_kernel")) return rc;
        }
        return 0;
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_predict(int64_t n, const int32_t *u, const int32_t *i, const void *pu, const void *bu,
               int32_t ldu, const void *qb, int32_t ldq, const void *imp, int32_t n_factors,
               int32_t biased, double global_mean, void *est, int32_t *impossible, int32_t dtype,
               void *stream)
{
    if (n <= 0) return 0;
    if (!u || !i || !pu || !bu || !qb || !est || !impossible)
        return set_err(MF_E_ARG, "null argument");
    if (n_factors < 0 || ldu < n_factors || ldq < n_factors + 1)
        return set_err(MF_E_ARG, "need ldu >= n_factors, ldq >= n_factors+1");
    const int64_t waves = default_waves(n);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T>(ldu, [&](auto vc) -> int {
            hipLaunchKernelGGL((predict_kernel<T, decltype(vc)::value>), dim3(grid_for_waves(waves)),
                               dim3(kBlock), 0, st, n, u, i, (const T *)pu, (const T *)bu, ldu,
                               (const T *)qb, ldq, (const T *)imp, n_factors, biased,
                               (T)global_mean, (T *)est, impossible);
            return check_launch("predict_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_rating_errors(int64_t n, const void *est, const int32_t *impossible, const void *r,
                     double fallback, double offset, double lo, double hi, double *out,
                     int32_t dtype, void *stream)
{
    if (n <= 0) return 0;
    if (!est || !r || !out) return set_err(MF_E_ARG, "null argument");
    int64_t b = (n + kBlock - 1) / kBlock;
    const int g = (int)(b > 2048 ? 2048 : b);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(rating_errors_kernel<float>, dim3(g), dim3(kBlock), 0, st, n,
                           (const float *)est, impossible, (const double *)r, fallback, offset,
                           lo, hi, out);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(rating_errors_kernel<double>, dim3(g), dim3(kBlock), 0, st, n,
                           (const double *)est, impossible, (const double *)r, fallback, offset,
                           lo, hi, out);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("rating_errors_kernel");
}

int mf_svdpp_user_implicit(const mf_csr_t *csr, const void *yj, int32_t ldu, void *imp,
                           int32_t n_factors, int32_t dtype, void *stream)
{
    if (!csr || !csr->row_ptr || !csr->items || !yj || !imp) return set_err(MF_E_ARG, "null argument");
    if (n_factors < 1 || ldu < n_factors) return set_err(MF_E_ARG, "need 1 <= n_factors <= ldu");
    if (csr->n_users <= 0) return 0;
    const int64_t waves = default_waves(csr->n_users);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T>(ldu, [&](auto vc) -> int {
            hipLaunchKernelGGL((user_implicit_kernel<T, decltype(vc)::value>),
                               dim3(grid_for_waves(waves)), dim3(kBlock), 0, st, csr->row_ptr,
                               csr->items, csr->n_users, (const T *)yj, ldu, (T *)imp, n_factors);
            return check_launch("user_implicit_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_xcd_layout(int32_t *ok)
{
    if (!ok) return set_err(MF_E_ARG, "null argument");
    *ok = xcd_layout_ok();
    return 0;
}

int mf_dispatch_check(uint64_t *sum)
{
    if (!sum) return set_err(MF_E_ARG, "null sum");
    // every code object's g_dispatch_sum: the main unit's (log replay, blocked solve) and each
    // epoch unit's; synchronous, after the device's work (hipMemcpyFromSymbol)
    unsigned long long total = 0, x = 0;
    int bad = dispatch_sum_here(&x);
    total += x;
    auto add = [&](auto tag_t) {
        using T = decltype(tag_t);
        bad |= mf_ext::dispatch_sum_tm<T, kPlain, false>(&x); total += x;
        bad |= mf_ext::dispatch_sum_tm<T, kPlain, true>(&x); total += x;
        bad |= mf_ext::dispatch_sum_tm<T, kAtomic, false>(&x); total += x;
        bad |= mf_ext::dispatch_sum_tm<T, kAtomic, true>(&x); total += x;
        bad |= mf_ext::dispatch_sum_tm<T, kLog, false>(&x); total += x;
        bad |= mf_ext::dispatch_sum_tm<T, kLog, true>(&x); total += x;
    };
    add(float{});
    add(double{});
    if (bad) return set_err((int)hipErrorInvalidSymbol, "mf_dispatch_check: hipMemcpyFromSymbol failed");
    *sum = total;
    return 0;
}

int mf_selftest_xcc(int32_t *out, int32_t n_blocks, void *stream)
{
    if (!out || n_blocks < 1) return set_err(MF_E_ARG, "bad argument");
    hipLaunchKernelGGL(xcc_selftest_kernel, dim3(n_blocks), dim3(kWave), 0, (hipStream_t)stream, out,
                       n_blocks);
    return check_launch("xcc_selftest_kernel");
}

int mf_selftest_wave_sum(const void *in, void *out, int32_t n_waves, int32_t dtype, void *stream)
{
    if (!in || !out || n_waves < 1) return set_err(MF_E_ARG, "bad argument");
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(wave_sum_selftest_kernel<float>, dim3(grid_for_waves(n_waves)),
                           dim3(kBlock), 0, st, (const float *)in, (float *)out, n_waves);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(wave_sum_selftest_kernel<double>, dim3(grid_for_waves(n_waves)),
                           dim3(kBlock), 0, st, (const double *)in, (double *)out, n_waves);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("wave_sum_selftest_kernel");
}

}  // extern "C"

#endif  // MF_TU_EPOCH

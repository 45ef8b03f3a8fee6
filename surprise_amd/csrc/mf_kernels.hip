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
//   * the user's (item, rating) stream is read in 64-entry chunks, one entry per lane, and the
//     next PF item rows are gathered ahead of use (software pipeline) so that the dependent
//     chain per rating is register-only: FMA partials -> DPP/permlane wave reduction -> error ->
//     FMA updates;
//   * the dot product is reduced with 4 DPP row ops + v_permlane16_swap + v_permlane32_swap
//     (no LDS round trip), leaving the sum in every lane.
// No MFMA: the path is gather/scatter-bound.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "../../include/surprise_amd.h"

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves per workgroup
constexpr int kPF = 8;       // item rows gathered ahead of use

thread_local char g_err[256] = "";

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

template <typename T>
struct Hyper {
    T lr_bu, lr_bi, lr_pu, lr_qi, lr_yj, reg_bu, reg_bi, reg_pu, reg_qi, reg_yj, gm;
};

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

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
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
    // HW_REG_XCC_ID (hwreg 20), bits [3:0]: the XCD this wave runs on. Used only to pick an
    // item-table replica (a speed/locality choice; any placement is correct).
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 0xF);
}

// Item-side loads bypass the CU's vector L1 (global_load ... sc1, served by the XCD's L2):
// the L1 is never refreshed by other CUs' stores, so a plain load of a hot item row can return
// a stale copy for a long time and the following store then erases other waves' updates.
template <typename T>
__device__ __forceinline__ T ld_l2(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__device__ __forceinline__ void atomic_add(T *p, T v) {
    atomicAdd(p, v);  // global_atomic_add_f32 / _f64, executed at the memory side (no CAS loop)
}

// The user's (item, rating) stream, read 64 entries per wave instruction (one per lane) and
// double-buffered: `cur` covers [base, base+64), `nxt` covers [base+64, base+128).
template <typename T>
struct RatingStream {
    const int32_t *items;
    const T *ratings;
    int64_t base;
    int i_cur, i_nxt;
    T r_cur, r_nxt;

    int64_t end;

    __device__ __forceinline__ void load(int64_t at, int lane, int &i, T &r) const {
        const int64_t k = at + lane;
        i = k < end ? items[k] : 0;
        r = k < end ? ratings[k] : T(0);
    }
    __device__ __forceinline__ void init(const int32_t *it, const T *rt, int64_t s, int64_t e,
                                         int lane) {
        items = it; ratings = rt; base = s; end = e;
        load(s, lane, i_cur, r_cur);
        load(s + 64, lane, i_nxt, r_nxt);
    }
    // entry k (base <= k < base + 128), uniform
    __device__ __forceinline__ int item(int64_t k) const {
        const int off = (int)(k - base);
        return off < 64 ? readlane(i_cur, off) : readlane(i_nxt, off - 64);
    }
    __device__ __forceinline__ T rating(int64_t k) const {
        const int off = (int)(k - base);
        return off < 64 ? readlane(r_cur, off) : readlane(r_nxt, off - 64);
    }
    // keep k_next within the window: slide by one chunk once k_next passes base + 64
    __device__ __forceinline__ void advance(int64_t k_next, int lane) {
        if (k_next - base >= 64) {
            base += 64;
            i_cur = i_nxt; r_cur = r_nxt;
            load(base + 64, lane, i_nxt, r_nxt);
        }
    }
};

// ---------------------------------------------------------------- SVD epoch kernel

enum { kPlain = MF_MODE_PLAIN, kAtomic = MF_MODE_ATOMIC, kReplica = MF_MODE_REPLICA };

template <typename T, int V, int MODE>
__global__ __launch_bounds__(kBlock) void svd_epoch_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, T *qi, T *bi, int K, int ld, int biased,
    Hyper<T> hp, int n_rep, int64_t rep_stride_q, int64_t rep_stride_b, int dups,
    int64_t n_waves_req)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int64_t grid_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t n_waves = n_waves_req < grid_waves ? n_waves_req : grid_waves;
    if (wave >= n_waves) return;  // whole wave exits (a 1-wave launch still uses a 4-wave block)

    T *q_tab = qi;
    T *b_tab = bi;
    if (MODE == kReplica) {
        const int rep = xcc_id() % n_rep;
        q_tab += rep * rep_stride_q;
        b_tab += rep * rep_stride_b;
    }
    bool fin[V];  // lane holds a real factor column for slot v
#pragma unroll
    for (int v = 0; v < V; ++v) fin[v] = lane + kWave * v < K;

    for (int64_t w = wave; w < n_sched; w += n_waves) {
        const int u = sched[w];
        const int64_t s = row_ptr[u], e = row_ptr[u + 1];
        if (s >= e) continue;

        T p[V];
#pragma unroll
        for (int v = 0; v < V; ++v) p[v] = fin[v] ? pu[(int64_t)u * ld + lane + kWave * v] : T(0);
        T bu_u = bu[u];

        RatingStream<T> rs;
        rs.init(items, ratings, s, e, lane);

        int s_i[kPF];
        T s_r[kPF], s_b[kPF], s_q[kPF][V];
        auto issue = [&](int slot, int64_t k) {
            const int i = rs.item(k);
            s_i[slot] = i;
            s_r[slot] = rs.rating(k);
            s_b[slot] = ld_l2(b_tab + i);
            const T *row = q_tab + (int64_t)i * ld + lane;
#pragma unroll
            for (int v = 0; v < V; ++v) s_q[slot][v] = fin[v] ? ld_l2(row + kWave * v) : T(0);
        };
#pragma unroll
        for (int d = 0; d < kPF; ++d)
            if (s + d < e) issue(d, s + d);

        for (int64_t t = s; t < e; t += kPF) {
#pragma unroll
            for (int d = 0; d < kPF; ++d) {
                const int64_t k = t + d;
                if (k >= e) break;
                const int i = s_i[d];
                const T r = s_r[d];
                const T b_old = s_b[d];
                // dot = <q_i, p_u>  (mf.pyx:247-249)
                T part = T(0);
#pragma unroll
                for (int v = 0; v < V; ++v) part += s_q[d][v] * p[v];
                const T dot = wave_sum(part);
                const T err = r - (hp.gm + bu_u + b_old + dot);  // mf.pyx:250
                T b_new = b_old;
                if (biased) {  // mf.pyx:253-255
                    bu_u += hp.lr_bu * (err - hp.reg_bu * bu_u);
                    b_new = b_old + hp.lr_bi * (err - hp.reg_bi * b_old);
                }
                T q_new[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {  // mf.pyx:258-262 (old puf, qif)
                    const T puf = p[v], qif = s_q[d][v];
                    p[v] = puf + hp.lr_pu * (err * qif - hp.reg_pu * puf);
                    q_new[v] = qif + hp.lr_qi * (err * puf - hp.reg_qi * qif);
                }
                T *row = q_tab + (int64_t)i * ld + lane;
                if (MODE == kAtomic) {
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (fin[v]) atomic_add(row + kWave * v, q_new[v] - s_q[d][v]);
                    if (biased && lane == 0) atomic_add(b_tab + i, b_new - b_old);
                } else {
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (fin[v]) row[kWave * v] = q_new[v];
                    if (biased && lane == 0) b_tab[i] = b_new;
                }
                // next gather for this slot
                const int64_t kn = k + kPF;
                if (kn < e) issue(d, kn);
                if (dups) {  // same item again within this user's window: forward the new row
#pragma unroll
                    for (int dd = 0; dd < kPF; ++dd) {
                        if (s_i[dd] == i && (dd != d || kn < e)) {
                            s_b[dd] = b_new;
#pragma unroll
                            for (int v = 0; v < V; ++v) s_q[dd][v] = q_new[v];
                        }
                    }
                }
            }
            rs.advance(t + 2 * kPF, lane);
        }
#pragma unroll
        for (int v = 0; v < V; ++v)
            if (fin[v]) pu[(int64_t)u * ld + lane + kWave * v] = p[v];
        if (lane == 0) bu[u] = bu_u;
    }
}

// ---------------------------------------------------------------- SVD++ epoch kernel

template <typename T, int V, int MODE>
__global__ __launch_bounds__(kBlock) void svdpp_epoch_kernel(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ items,
    const T *__restrict__ ratings, const int32_t *__restrict__ sched, int64_t n_sched,
    T *__restrict__ pu, T *__restrict__ bu, T *qi, T *bi, T *yj, int K, int ld, Hyper<T> hp,
    int n_rep, int64_t rep_stride_q, int64_t rep_stride_b, int dups, int64_t n_waves_req)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int64_t grid_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    const int64_t n_waves = n_waves_req < grid_waves ? n_waves_req : grid_waves;
    if (wave >= n_waves) return;

    T *q_tab = qi, *y_tab = yj, *b_tab = bi;
    if (MODE == kReplica) {
        const int rep = xcc_id() % n_rep;
        q_tab += rep * rep_stride_q;
        y_tab += rep * rep_stride_q;
        b_tab += rep * rep_stride_b;
    }
    bool fin[V];
#pragma unroll
    for (int v = 0; v < V; ++v) fin[v] = lane + kWave * v < K;
    const T decay = T(1) - hp.lr_yj * hp.reg_yj;

    for (int64_t w = wave; w < n_sched; w += n_waves) {
        const int u = sched[w];
        const int64_t s = row_ptr[u], e = row_ptr[u + 1];
        if (s >= e) continue;
        const T sqrt_n = sqrt(T(e - s));  // mf.pyx:470

        // 1) u_impl = sum_j y_j / sqrt|I_u|   (mf.pyx:473-476, same per-term division)
        T imp[V];
#pragma unroll
        for (int v = 0; v < V; ++v) imp[v] = T(0);
        for (int64_t c0 = s; c0 < e; c0 += kWave) {
            const int jl = c0 + lane < e ? items[c0 + lane] : 0;
            const int cnt = e - c0 < kWave ? (int)(e - c0) : kWave;
            int x = 0;
            for (; x + 8 <= cnt; x += 8) {
                T g[8][V];
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    const T *row = y_tab + (int64_t)readlane(jl, x + a) * ld + lane;
#pragma unroll
                    for (int v = 0; v < V; ++v) g[a][v] = fin[v] ? ld_l2(row + kWave * v) : T(0);
                }
#pragma unroll
                for (int a = 0; a < 8; ++a)
#pragma unroll
                    for (int v = 0; v < V; ++v) imp[v] += g[a][v] / sqrt_n;
            }
            for (; x < cnt; ++x) {
                const T *row = y_tab + (int64_t)readlane(jl, x) * ld + lane;
#pragma unroll
                for (int v = 0; v < V; ++v) imp[v] += (fin[v] ? ld_l2(row + kWave * v) : T(0)) / sqrt_n;
            }
        }

        // 2) the user's ratings in order, y_j kept implicit as y_j(start)*A + c
        T p[V], cacc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            p[v] = fin[v] ? pu[(int64_t)u * ld + lane + kWave * v] : T(0);
            cacc[v] = T(0);
        }
        T bu_u = bu[u];
        T A = T(1);

        RatingStream<T> rs;
        rs.init(items, ratings, s, e, lane);
        int s_i[kPF];
        T s_r[kPF], s_b[kPF], s_q[kPF][V];
        auto issue = [&](int slot, int64_t k) {
            const int i = rs.item(k);
            s_i[slot] = i;
            s_r[slot] = rs.rating(k);
            s_b[slot] = ld_l2(b_tab + i);
            const T *row = q_tab + (int64_t)i * ld + lane;
#pragma unroll
            for (int v = 0; v < V; ++v) s_q[slot][v] = fin[v] ? ld_l2(row + kWave * v) : T(0);
        };
#pragma unroll
        for (int d = 0; d < kPF; ++d)
            if (s + d < e) issue(d, s + d);

        for (int64_t t = s; t < e; t += kPF) {
#pragma unroll
            for (int d = 0; d < kPF; ++d) {
                const int64_t k = t + d;
                if (k >= e) break;
                const int i = s_i[d];
                const T r = s_r[d];
                const T b_old = s_b[d];
                T part = T(0);  // mf.pyx:479-481
#pragma unroll
                for (int v = 0; v < V; ++v) part += s_q[d][v] * (p[v] + imp[v]);
                const T dot = wave_sum(part);
                const T err = r - (hp.gm + bu_u + b_old + dot);  // mf.pyx:483
                bu_u += hp.lr_bu * (err - hp.reg_bu * bu_u);     // mf.pyx:486-487
                const T b_new = b_old + hp.lr_bi * (err - hp.reg_bi * b_old);
                T q_new[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {  // mf.pyx:490-498
                    const T puf = p[v], qif = s_q[d][v];
                    p[v] = puf + hp.lr_pu * (err * qif - hp.reg_pu * puf);
                    q_new[v] = qif + hp.lr_qi * (err * (puf + imp[v]) - hp.reg_qi * qif);
                    cacc[v] = decay * cacc[v] + hp.lr_yj * (err * qif / sqrt_n);
                    imp[v] = decay * imp[v] + hp.lr_yj * err * qif;
                }
                A *= decay;
                T *row = q_tab + (int64_t)i * ld + lane;
                if (MODE == kAtomic) {
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (fin[v]) atomic_add(row + kWave * v, q_new[v] - s_q[d][v]);
                    if (lane == 0) atomic_add(b_tab + i, b_new - b_old);
                } else {
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (fin[v]) row[kWave * v] = q_new[v];
                    if (lane == 0) b_tab[i] = b_new;
                }
                const int64_t kn = k + kPF;
                if (kn < e) issue(d, kn);
                if (dups) {
#pragma unroll
                    for (int dd = 0; dd < kPF; ++dd) {
                        if (s_i[dd] == i && (dd != d || kn < e)) {
                            s_b[dd] = b_new;
#pragma unroll
                            for (int v = 0; v < V; ++v) s_q[dd][v] = q_new[v];
                        }
                    }
                }
            }
            rs.advance(t + 2 * kPF, lane);
        }
#pragma unroll
        for (int v = 0; v < V; ++v)
            if (fin[v]) pu[(int64_t)u * ld + lane + kWave * v] = p[v];
        if (lane == 0) bu[u] = bu_u;

        // 3) y_j <- A y_j + c  for every j in I_u
        for (int64_t c0 = s; c0 < e; c0 += kWave) {
            const int jl = c0 + lane < e ? items[c0 + lane] : 0;
            const int cnt = e - c0 < kWave ? (int)(e - c0) : kWave;
            int x = 0;
            for (; x + 8 <= cnt; x += 8) {
                T g[8][V];
                T *rows[8];
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    rows[a] = y_tab + (int64_t)readlane(jl, x + a) * ld + lane;
#pragma unroll
                    for (int v = 0; v < V; ++v) g[a][v] = fin[v] ? ld_l2(rows[a] + kWave * v) : T(0);
                }
#pragma unroll
                for (int a = 0; a < 8; ++a)
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        if (!fin[v]) continue;
                        if (MODE == kAtomic)
                            atomic_add(rows[a] + kWave * v, (A - T(1)) * g[a][v] + cacc[v]);
                        else
                            rows[a][kWave * v] = A * g[a][v] + cacc[v];
                    }
            }
            for (; x < cnt; ++x) {
                T *row = y_tab + (int64_t)readlane(jl, x) * ld + lane;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    if (!fin[v]) continue;
                    const T y = ld_l2(row + kWave * v);
                    if (MODE == kAtomic)
                        atomic_add(row + kWave * v, (A - T(1)) * y + cacc[v]);
                    else
                        row[kWave * v] = A * y + cacc[v];
                }
            }
        }
    }
}

// ---------------------------------------------------------------- merge / apply (elementwise)

struct SegDesc {
    void *ptr[8];
    void *snap[8];
    int64_t len[8];
    int64_t stride[8];
    int64_t off[9];  // packed offsets into delta
    int n_seg;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void merge_kernel(SegDesc d, int n_rep, T *delta, int apply)
{
    const int64_t total = d.off[d.n_seg];
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total; x += step) {
        int sg = 0;
        while (sg + 1 < d.n_seg && x >= d.off[sg + 1]) ++sg;
        const int64_t j = x - d.off[sg];
        T *base = (T *)d.ptr[sg];
        T *snap = (T *)d.snap[sg];
        const T s0 = snap[j];
        T acc = T(0);
        for (int r = 0; r < n_rep; ++r) acc += base[r * d.stride[sg] + j] - s0;
        if (apply) {
            const T nv = s0 + acc;
            snap[j] = nv;
            for (int r = 0; r < n_rep; ++r) base[r * d.stride[sg] + j] = nv;
        }
        if (delta) delta[x] = acc;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void apply_kernel(SegDesc d, int n_rep, const T *delta)
{
    const int64_t total = d.off[d.n_seg];
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total; x += step) {
        int sg = 0;
        while (sg + 1 < d.n_seg && x >= d.off[sg + 1]) ++sg;
        const int64_t j = x - d.off[sg];
        T *base = (T *)d.ptr[sg];
        T *snap = (T *)d.snap[sg];
        const T nv = snap[j] + delta[x];
        snap[j] = nv;
        for (int r = 0; r < n_rep; ++r) base[r * d.stride[sg] + j] = nv;
    }
}

// ---------------------------------------------------------------- inference

template <typename T, int V>
__global__ __launch_bounds__(kBlock) void predict_kernel(
    int64_t n, const int32_t *__restrict__ uu, const int32_t *__restrict__ ii,
    const T *__restrict__ pu, const T *__restrict__ qi, const T *__restrict__ bu,
    const T *__restrict__ bi, const T *__restrict__ imp, int K, int ld, int biased, T gm,
    T *__restrict__ est, int32_t *__restrict__ impossible)
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
                    T pf = pu[(int64_t)u * ld + f];
                    if (imp) pf += imp[(int64_t)u * ld + f];
                    part += qi[(int64_t)i * ld + f] * pf;
                }
            }
        }
        const T dot = wave_sum(part);
        if (lane == 0) {
            int bad = 0;
            T e;
            if (biased) {
                e = gm;
                if (ku) e += bu[u];
                if (ki) e += bi[i];
                if (ku && ki) e += dot;
            } else if (ku && ki) {
                e = dot;
            } else {
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
    const T *__restrict__ yj, T *__restrict__ imp, int K, int ld)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int64_t n_waves = ((int64_t)gridDim.x * kBlock) / kWave;
    for (int64_t u = wave; u < n_users; u += n_waves) {
        const int64_t s = row_ptr[u], e = row_ptr[u + 1];
        T acc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = T(0);
        for (int64_t k = s; k < e; ++k) {
            const T *row = yj + (int64_t)items[k] * ld + lane;
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (lane + kWave * v < K) acc[v] += row[kWave * v];
        }
        const T sq = sqrt(T(e - s));
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int f = lane + kWave * v;
            if (f < ld) imp[u * ld + f] = (e > s && f < K) ? acc[v] / sq : T(0);
        }
    }
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

int grid_for_waves(int64_t waves) {
    int64_t blocks = (waves * kWave + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

// Default grid: enough waves to hold every scheduled user, capped at 16 waves per CU.
int64_t default_waves(int64_t n_sched) {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            n_cu = prop.multiProcessorCount;
        if (n_cu <= 0) n_cu = 256;
    }
    const int64_t cap = (int64_t)n_cu * 16;
    return n_sched < cap ? n_sched : cap;
}

template <typename T, int V, int MODE>
int launch_svd_v(const mf_csr_t *c, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                 void *qi, void *bi, int K, int ld, int biased, const mf_hyper_t *hp, int n_rep,
                 int64_t rsq, int64_t rsb, int64_t waves, int dups, hipStream_t st)
{
    hipLaunchKernelGGL((svd_epoch_kernel<T, V, MODE>), dim3(grid_for_waves(waves)), dim3(kBlock), 0,
                       st, c->row_ptr, c->items, (const T *)c->ratings, sched, n_sched, (T *)pu,
                       (T *)bu, (T *)qi, (T *)bi, K, ld, biased, cast_hyper<T>(hp), n_rep, rsq, rsb,
                       dups, waves);
    return check_launch("svd_epoch_kernel");
}

template <typename T, int V, int MODE>
int launch_svdpp_v(const mf_csr_t *c, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                   void *qi, void *bi, void *yj, int K, int ld, const mf_hyper_t *hp, int n_rep,
                   int64_t rsq, int64_t rsb, int64_t waves, int dups, hipStream_t st)
{
    hipLaunchKernelGGL((svdpp_epoch_kernel<T, V, MODE>), dim3(grid_for_waves(waves)), dim3(kBlock),
                       0, st, c->row_ptr, c->items, (const T *)c->ratings, sched, n_sched,
                       (T *)pu, (T *)bu, (T *)qi, (T *)bi, (T *)yj, K, ld, cast_hyper<T>(hp),
                       n_rep, rsq, rsb, dups, waves);
    return check_launch("svdpp_epoch_kernel");
}

// V = elements per lane = ceil(ld / 64)
template <typename T, int MODE, typename F>
int dispatch_v(int ld, F &&f)
{
    const int v = (ld + kWave - 1) / kWave;
    if (v <= 1) return f(std::integral_constant<int, 1>{});
    if (v <= 2) return f(std::integral_constant<int, 2>{});
    if (v <= 4) return f(std::integral_constant<int, 4>{});
    if (sizeof(T) == 4 && v <= 8) return f(std::integral_constant<int, 8>{});
    return set_err(MF_E_ARG, "n_factors/ld too large");
}

int check_common(const mf_csr_t *c, int K, int ld, int mode, int n_rep, int dtype)
{
    if (!c || !c->row_ptr || !c->items || !c->ratings) return set_err(MF_E_ARG, "null csr");
    if (K < 1 || ld < K) return set_err(MF_E_ARG, "need 1 <= n_factors <= ld");
    if (dtype == MF_F32 && ld > MF_MAX_FACTORS_F32) return set_err(MF_E_ARG, "ld > 512 (f32)");
    if (dtype == MF_F64 && ld > MF_MAX_FACTORS_F64) return set_err(MF_E_ARG, "ld > 256 (f64)");
    if (dtype != MF_F32 && dtype != MF_F64) return set_err(MF_E_ARG, "bad dtype");
    if (mode < MF_MODE_PLAIN || mode > MF_MODE_REPLICA) return set_err(MF_E_ARG, "bad mode");
    if (mode == MF_MODE_REPLICA && (n_rep < 1 || n_rep > 16))
        return set_err(MF_E_ARG, "n_replicas must be in [1, 16]");
    return 0;
}

int build_segs(SegDesc &d, int n_seg, void *const *ptr, void *const *snap, const int64_t *len,
               const int64_t *stride)
{
    if (n_seg < 1 || n_seg > 8) return set_err(MF_E_ARG, "n_seg must be in [1, 8]");
    d.n_seg = n_seg;
    d.off[0] = 0;
    for (int s = 0; s < n_seg; ++s) {
        d.ptr[s] = ptr[s];
        d.snap[s] = snap[s];
        d.len[s] = len[s];
        d.stride[s] = stride[s];
        d.off[s + 1] = d.off[s] + len[s];
    }
    for (int s = n_seg; s < 8; ++s) {
        d.ptr[s] = d.snap[s] = nullptr;
        d.len[s] = d.stride[s] = 0;
        d.off[s + 1] = d.off[s];
    }
    return 0;
}

int elementwise_grid(int64_t total) {
    int64_t b = (total + kBlock - 1) / kBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace

extern "C" {

int mf_version(void) { return 100; }

const char *mf_last_error(void) { return g_err; }

int mf_svd_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                 void *qi, void *bi, int32_t n_factors, int32_t ld, int32_t biased,
                 const mf_hyper_t *hp, int32_t mode, int32_t n_replicas, int64_t rep_stride_q,
                 int64_t rep_stride_b, int32_t n_waves, int32_t dup_items, int32_t dtype,
                 void *stream)
{
    if (int rc = check_common(csr, n_factors, ld, mode, n_replicas, dtype)) return rc;
    if (!hp || !sched || !pu || !bu || !qi || !bi) return set_err(MF_E_ARG, "null argument");
    if (n_sched <= 0) return 0;
    const int64_t waves = n_waves > 0 ? n_waves : default_waves(n_sched);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t, auto mode_c) -> int {
        using T = decltype(tag_t);
        constexpr int M = decltype(mode_c)::value;
        return dispatch_v<T, M>(ld, [&](auto vc) -> int {
            return launch_svd_v<T, decltype(vc)::value, M>(csr, sched, n_sched, pu, bu, qi, bi,
                                                          n_factors, ld, biased, hp, n_replicas,
                                                          rep_stride_q, rep_stride_b, waves,
                                                          dup_items, st);
        });
    };
    auto by_mode = [&](auto tag_t) -> int {
        switch (mode) {
            case MF_MODE_PLAIN: return run(tag_t, std::integral_constant<int, kPlain>{});
            case MF_MODE_ATOMIC: return run(tag_t, std::integral_constant<int, kAtomic>{});
            default: return run(tag_t, std::integral_constant<int, kReplica>{});
        }
    };
    return dtype == MF_F32 ? by_mode(float{}) : by_mode(double{});
}

int mf_svdpp_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                   void *qi, void *bi, void *yj, int32_t n_factors, int32_t ld,
                   const mf_hyper_t *hp, int32_t mode, int32_t n_replicas, int64_t rep_stride_q,
                   int64_t rep_stride_b, int32_t n_waves, int32_t dup_items, int32_t dtype,
                   void *stream)
{
    if (int rc = check_common(csr, n_factors, ld, mode, n_replicas, dtype)) return rc;
    if (!hp || !sched || !pu || !bu || !qi || !bi || !yj) return set_err(MF_E_ARG, "null argument");
    if (n_sched <= 0) return 0;
    const int64_t waves = n_waves > 0 ? n_waves : default_waves(n_sched);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t, auto mode_c) -> int {
        using T = decltype(tag_t);
        constexpr int M = decltype(mode_c)::value;
        return dispatch_v<T, M>(ld, [&](auto vc) -> int {
            return launch_svdpp_v<T, decltype(vc)::value, M>(csr, sched, n_sched, pu, bu, qi, bi,
                                                            yj, n_factors, ld, hp, n_replicas,
                                                            rep_stride_q, rep_stride_b, waves,
                                                            dup_items, st);
        });
    };
    auto by_mode = [&](auto tag_t) -> int {
        switch (mode) {
            case MF_MODE_PLAIN: return run(tag_t, std::integral_constant<int, kPlain>{});
            case MF_MODE_ATOMIC: return run(tag_t, std::integral_constant<int, kAtomic>{});
            default: return run(tag_t, std::integral_constant<int, kReplica>{});
        }
    };
    return dtype == MF_F32 ? by_mode(float{}) : by_mode(double{});
}

int mf_replica_merge(int32_t n_seg, void *const *seg_ptr, void *const *seg_snap,
                     const int64_t *seg_len, const int64_t *seg_stride, int32_t n_replicas,
                     void *delta_out, int32_t apply, int32_t dtype, void *stream)
{
    SegDesc d;
    if (int rc = build_segs(d, n_seg, seg_ptr, seg_snap, seg_len, seg_stride)) return rc;
    if (n_replicas < 1) return set_err(MF_E_ARG, "n_replicas < 1");
    if (!delta_out && !apply) return 0;
    const int g = elementwise_grid(d.off[n_seg]);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(merge_kernel<float>, dim3(g), dim3(kBlock), 0, st, d, n_replicas,
                           (float *)delta_out, apply);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(merge_kernel<double>, dim3(g), dim3(kBlock), 0, st, d, n_replicas,
                           (double *)delta_out, apply);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("merge_kernel");
}

int mf_apply_delta(int32_t n_seg, void *const *seg_ptr, void *const *seg_snap,
                   const int64_t *seg_len, const int64_t *seg_stride, int32_t n_replicas,
                   const void *delta, int32_t dtype, void *stream)
{
    SegDesc d;
    if (int rc = build_segs(d, n_seg, seg_ptr, seg_snap, seg_len, seg_stride)) return rc;
    if (!delta || n_replicas < 1) return set_err(MF_E_ARG, "null delta / n_replicas < 1");
    const int g = elementwise_grid(d.off[n_seg]);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MF_F32)
        hipLaunchKernelGGL(apply_kernel<float>, dim3(g), dim3(kBlock), 0, st, d, n_replicas,
                           (const float *)delta);
    else if (dtype == MF_F64)
        hipLaunchKernelGGL(apply_kernel<double>, dim3(g), dim3(kBlock), 0, st, d, n_replicas,
                           (const double *)delta);
    else
        return set_err(MF_E_ARG, "bad dtype");
    return check_launch("apply_kernel");
}

int mf_predict(int64_t n, const int32_t *u, const int32_t *i, const void *pu, const void *qi,
               const void *bu, const void *bi, const void *imp, int32_t n_factors, int32_t ld,
               int32_t biased, double global_mean, void *est, int32_t *impossible, int32_t dtype,
               void *stream)
{
    if (n <= 0) return 0;
    if (!u || !i || !pu || !qi || !bu || !bi || !est || !impossible)
        return set_err(MF_E_ARG, "null argument");
    if (n_factors < 1 || ld < n_factors) return set_err(MF_E_ARG, "need 1 <= n_factors <= ld");
    const int64_t waves = default_waves(n);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T, 0>(ld, [&](auto vc) -> int {
            hipLaunchKernelGGL((predict_kernel<T, decltype(vc)::value>), dim3(grid_for_waves(waves)),
                               dim3(kBlock), 0, st, n, u, i, (const T *)pu, (const T *)qi,
                               (const T *)bu, (const T *)bi, (const T *)imp, n_factors, ld, biased,
                               (T)global_mean, (T *)est, impossible);
            return check_launch("predict_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
}

int mf_svdpp_user_implicit(const mf_csr_t *csr, const void *yj, void *imp, int32_t n_factors,
                           int32_t ld, int32_t dtype, void *stream)
{
    if (!csr || !csr->row_ptr || !csr->items || !yj || !imp) return set_err(MF_E_ARG, "null argument");
    if (n_factors < 1 || ld < n_factors) return set_err(MF_E_ARG, "need 1 <= n_factors <= ld");
    if (csr->n_users <= 0) return 0;
    const int64_t waves = default_waves(csr->n_users);
    hipStream_t st = (hipStream_t)stream;
    auto run = [&](auto tag_t) -> int {
        using T = decltype(tag_t);
        return dispatch_v<T, 0>(ld, [&](auto vc) -> int {
            hipLaunchKernelGGL((user_implicit_kernel<T, decltype(vc)::value>),
                               dim3(grid_for_waves(waves)), dim3(kBlock), 0, st, csr->row_ptr,
                               csr->items, csr->n_users, (const T *)yj, (T *)imp, n_factors, ld);
            return check_launch("user_implicit_kernel");
        });
    };
    if (dtype == MF_F32) return run(float{});
    if (dtype == MF_F64) return run(double{});
    return set_err(MF_E_ARG, "bad dtype");
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

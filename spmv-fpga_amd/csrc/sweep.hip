// Kernel 2 — "panel sweep": the reference's 2-D blocking turned around for MI355X.
//
// The reference keeps a whole column block of x in every CU's BRAM and streams that block's
// rows through the CU, scattering each CU's compact y back on the host (spmv.cpp:169-205,
// csr_hw.cpp:1531-1565). For a matrix whose columns are spread at random over an x far larger
// than the 4 MiB L2 of an XCD, gathering x straight from HBM/Infinity Cache costs one L2 miss
// per non-zero, and MI355X serves only ~55 G such misses/s (tools/hbm_calib, profiles/).
// Here each workgroup instead owns a row panel whose y stays resident in LDS (<= 160 KiB) and
// walks the panel's non-zeros in ascending column order. All panels sweep the columns at the
// same pace, so the x lines in use at any moment form a narrow window that the XCD's L2 serves
// (~265 G gathers/s, 5x the miss rate). Products are accumulated with LDS fp64 atomics; y is
// written once per panel with coalesced stores. Bound: the L2 request rate (the L2 channels are
// busy 97 % of the kernel on the 10M/160M matrix), at ~0.8 x-line requests per
// non-zero for panels of 20K rows.
//
// Representation (built on the GPU in O(nnz) with a hipcub radix sort on 32-bit keys):
//   s_col u32[ent_pad]  column of each entry, panels contiguous, ascending column per panel
//   s_row u16[ent_pad]  row inside the panel (padding entries use the scratch slot R_p)
//   s_val V[ent_pad]    value
//   panel_row u32[P+1]  row range of panel p
//   unit_ent u32[U+1]   entry range of work unit u (a piece of whole chunks of one panel; a
//                       panel's pieces are consecutive units); one piece = the whole panel
//   unit_panel u32[U]   panel of unit u;  panel_unit u32[P+1]  first unit of each panel
// Packed form (default when every 128-entry chunk spans < 65536 columns, 12 B/entry):
//   s_col u32 holds (row_in_panel << 16) | (column - s_cbase[chunk]); s_row is dropped; inside a
//   chunk, word 2l+j holds entry 64j+l (k_sweep_lane_order) so one gather instruction covers 64
//   consecutive columns-sorted entries.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <tuple>
#include <cmath>
#include <cstring>

#include "spmv_internal.hpp"

namespace spmvhw {

// LDS accumulator A: fp64 (ds_add_f64) for both precisions by default; fp32 products are exact
// in fp64, so y of an fp32 matrix is the fp64 sum rounded once. An fp32 accumulator would let a
// panel hold twice the rows (40,895 instead of 20,447: denser panels), but gfx950 executes the
// native ds_add_f32 ~8x slower than ds_add_f64 at random rows (203 vs 1660 G adds/s,
// tools/lds_atomics.hip). A compare-and-swap loop on the float's bits matches ds_add_f64 in
// that microbenchmark, and env SPMV_SWEEP_ACC=32 selects it here; on the 10M/160M fp32 matrix
// it measured 1.94 ms against 0.60 ms for the fp64 accumulator (the CAS round trips serialise
// each wave: 1.04 ms without any gathers; profiles/r01_ab_variants.jsonl, session r01c_acc).
__device__ __forceinline__ void lds_add(double *p, double v) { atomicAdd(p, v); }
__device__ __forceinline__ void lds_add(float *p, float v)
{
    uint32_t *u = reinterpret_cast<uint32_t *>(p);
    uint32_t old = *u, assumed;
    do {
        assumed = old;
        old = atomicCAS(u, assumed, __float_as_uint(__uint_as_float(assumed) + v));
    } while (old != assumed);
}

// N adds of one lane at once: fp64 = N fire-and-forget ds_add_f64; fp32 = N reads, then N
// compare-and-swaps in flight together, then a retry loop for the (rare) ones another lane or
// wave got in between -- two LDS round trips per batch instead of two per add
template <int N>
__device__ __forceinline__ void lds_add_n(double *y, const uint32_t (&idx)[N], const double (&v)[N])
{
#pragma unroll
    for (int i = 0; i < N; ++i)
        atomicAdd(&y[idx[i]], v[i]);
}
template <int N>
__device__ __forceinline__ void lds_add_n(float *y, const uint32_t (&idx)[N], const float (&v)[N])
{
    uint32_t *u = reinterpret_cast<uint32_t *>(y);
    uint32_t old[N], got[N];
#pragma unroll
    for (int i = 0; i < N; ++i)
        old[i] = __hip_atomic_load(&u[idx[i]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int i = 0; i < N; ++i)
        got[i] = atomicCAS(&u[idx[i]], old[i], __float_as_uint(__uint_as_float(old[i]) + v[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) {
        while (got[i] != old[i]) {
            old[i] = got[i];
            got[i] = atomicCAS(&u[idx[i]], old[i], __float_as_uint(__uint_as_float(old[i]) + v[i]));
        }
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT, typename T>
__device__ __forceinline__ T lds_(const T *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT>
__device__ __forceinline__ void load4(const double *__restrict__ v, uint64_t e, double (&o)[4])
{
    const f64x2 a = lds_<NT>(reinterpret_cast<const f64x2 *>(v + e));
    const f64x2 b = lds_<NT>(reinterpret_cast<const f64x2 *>(v + e + 2));
    o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
template <bool NT>
__device__ __forceinline__ void load4(const float *__restrict__ v, uint64_t e, float (&o)[4])
{
    const f32x4 a = lds_<NT>(reinterpret_cast<const f32x4 *>(v + e));
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
}

template <int E> struct EntryVec;
template <> struct EntryVec<4> { typedef u32x4 C; typedef u16x4 R; };
template <> struct EntryVec<1> {
    typedef uint32_t C __attribute__((ext_vector_type(1)));
    typedef uint16_t R __attribute__((ext_vector_type(1)));
};
template <> struct EntryVec<2> {
    typedef uint32_t C __attribute__((ext_vector_type(2)));
    typedef uint16_t R __attribute__((ext_vector_type(2)));
};

template <bool NT, int E, typename V>
__device__ __forceinline__ void loadv(const V *__restrict__ v, uint64_t e, V (&o)[E])
{
    if constexpr (E == 4) {
        load4<NT>(v, e, o);
    } else if constexpr (E == 1) {
        o[0] = lds_<NT>(v + e);
    } else if constexpr (sizeof(V) == 8) {
        const f64x2 a = lds_<NT>(reinterpret_cast<const f64x2 *>(v + e));
        o[0] = a.x; o[1] = a.y;
    } else {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 a = lds_<NT>(reinterpret_cast<const f32x2 *>(v + e));
        o[0] = a.x; o[1] = a.y;
    }
}

// A unit's y: stored when the panel is one unit; a panel cut into pieces has each piece store
// its fp64 partial sums (its column range) into part[unit * stride + i]. The pieces of a panel
// are then added per row in piece order (deterministic, one rounding) -- by k_sweep_combine, a
// second kernel (default), or (pcnt != null, env SPMV_SWEEP_COMBINE=fused) by the piece that
// finishes last: each piece
// publishes its partials (agent-scope release: they leave its XCD's L2), bumps the panel's
// counter, and the one that sees pieces - 1 acquires, sums every piece's partials in piece order
// and stores y, then re-arms the counter for the next launch (runs of one plan are ordered). The
// sums are those of k_sweep_combine, bit for bit. It saves the second launch but serialises the
// slab reads on one workgroup per panel: slower here (see build_sweep).
template <typename V, int T, typename A>
__device__ __forceinline__ void write_panel(const A *__restrict__ ylds, uint32_t R, V *__restrict__ y,
                                            uint32_t pieces, A *__restrict__ part, uint32_t stride,
                                            uint32_t u0, uint32_t *__restrict__ pcnt)
{
    if (pieces == 1) {
        for (uint32_t i = threadIdx.x; i < R; i += T)
            y[i] = V(ylds[i]);
        return;
    }
    A *dst = part + (uint64_t)blockIdx.x * stride;
    for (uint32_t i = threadIdx.x; i < R; i += T)
        dst[i] = ylds[i];
    if (!pcnt)
        return;
    // the hand-off of cdna_hip_programming.md (in-launch split-K reduction): every wave drains its
    // stores, one lane releases at agent scope (the XCD L2's dirty lines written back) and draws
    // the ticket; the last arriver's lane 0 acquires, then all waves read the slabs
    __shared__ uint32_t last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pieces - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last)
        return;
    const A *src = part + (uint64_t)u0 * stride;
    for (uint32_t i = threadIdx.x; i < R; i += T) {
        A acc = src[i];
        for (uint32_t t = 1; t < pieces; ++t)
            acc += src[(uint64_t)t * stride + i];
        y[i] = V(acc);
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// y[r0 + i] = sum over the panel's pieces u (in order) of part[u * stride + i]; panels of one
// piece were written by the sweep itself
// steal != null: also re-arms the panel's work-stealing counters for the next launch
template <typename V, typename A>
__global__ __launch_bounds__(256) void k_sweep_combine(const uint32_t *__restrict__ panel_row,
                                                       const uint32_t *__restrict__ panel_unit,
                                                       const A *__restrict__ part, uint32_t stride,
                                                       V *__restrict__ y, unsigned long long *__restrict__ steal)
{
    const uint32_t p = blockIdx.y;
    const uint32_t u0 = panel_unit[p], u1 = panel_unit[p + 1];
    if (steal && blockIdx.x == 0)
        for (uint32_t t = threadIdx.x; t < u1 - u0; t += 256)
            steal[u0 + t] = 0;
    const uint32_t r0 = panel_row[p], R = panel_row[p + 1] - r0;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (u1 - u0 < 2 || i >= R)
        return;
    const A *src = part + (uint64_t)u0 * stride + i;
    A acc = src[0];
    for (uint32_t t = 1; t < u1 - u0; ++t)
        acc += src[(uint64_t)t * stride];
    y[r0 + i] = V(acc);
}

// E entries per thread per workgroup iteration, Q such groups per iteration; SYNC: barrier after
// every iteration so the 16 waves stay on one column window; NT: non-temporal entry loads.
// Entry ranges of a panel are multiples of 4, so whole E-groups are always valid.
template <typename V, int T, int E, int Q, bool SYNC, bool NT, typename A = double>
__global__ __launch_bounds__(T) void k_spmv_sweep(
    const uint32_t *__restrict__ col, const uint16_t *__restrict__ row, const V *__restrict__ val,
    const uint32_t *__restrict__ panel_row, const uint32_t *__restrict__ unit_ent,
    const uint32_t *__restrict__ unit_panel, const uint32_t *__restrict__ panel_unit,
    A *__restrict__ part, uint32_t stride, uint32_t *__restrict__ pcnt, const V *__restrict__ x,
    V *__restrict__ y)
{
    typedef typename EntryVec<E>::C CV;
    typedef typename EntryVec<E>::R RV;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    A *ylds = reinterpret_cast<A *>(smem);
    const uint32_t p = unit_panel[blockIdx.x];  // unit = a piece of a panel's column-sorted entries
    const uint32_t pieces = panel_unit[p + 1] - panel_unit[p];
    const uint32_t r0 = panel_row[p], R = panel_row[p + 1] - r0;
    const uint64_t e0 = unit_ent[blockIdx.x], e1 = unit_ent[blockIdx.x + 1];
    for (uint32_t i = threadIdx.x; i <= R; i += T)
        ylds[i] = A(0);
    __syncthreads();
    constexpr uint64_t kGroup = (uint64_t)E * T;  // entries per workgroup group
    // branch-free body (see k_spmv_sweep_packed): out-of-range groups re-read the panel's last
    // E entries and add into the scratch slot R
    const uint64_t elast = e1 > e0 ? e1 - E : e0;
    for (uint64_t base = e0; base < e1; base += Q * kGroup) {
        CV c[Q];
        RV r[Q];
        V v[Q][E];
        bool ok[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            uint64_t e = base + q * kGroup + (uint64_t)E * threadIdx.x;
            ok[q] = e < e1;
            e = ok[q] ? e : elast;
            c[q] = lds_<NT>(reinterpret_cast<const CV *>(col + e));
            r[q] = lds_<NT>(reinterpret_cast<const RV *>(row + e));
            loadv<NT, E>(val, e, v[q]);
        }
        V xv[Q][E];
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int j = 0; j < E; ++j)
                xv[q][j] = x[c[q][j]];
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int j = 0; j < E; ++j)
                lds_add(&ylds[ok[q] ? (uint32_t)r[q][j] : R], A(v[q][j]) * A(xv[q][j]));
        if constexpr (SYNC)
            __syncthreads();
    }
    __syncthreads();
    write_panel<V, T, A>(ylds, R, y + r0, pieces, part, stride, panel_unit[p], pcnt ? pcnt + p : nullptr);
}

// Packed entries (12 B instead of 14 B): rc = (row_in_panel << 16) | (column - chunk_base),
// one u32 base column per 128-entry chunk (one wave instruction of 2-entry lanes). Panels are
// padded to whole chunks, so the chunk of a wave is wave-uniform and its base is a scalar load.
// LAG = 0: one workgroup barrier per iteration. LAG = k > 0: no barrier; each wave publishes
// its iteration count in LDS and only waits (s_sleep) while it is more than k iterations
// ahead of the slowest wave, so the vector-memory pipe never drains at a common barrier.
// DL: delta-coded columns (11 B/entry fp64, 7 fp32): per entry a u16 row word and a u8, which
// together hold the row (15 bits) and a 9-bit column delta from the previous entry of the same
// wave instruction; a chunk's first entry counts from the chunk base dbase[c]. A 64-lane DPP
// prefix sum turns the deltas into columns. A chunk with a gap above 511 (~1 in 10^5 on the
// headline matrix) has bit 31 of dbase set and its absolute columns in `side` (uniform branch).
// `rc` is not read (a delta plan frees its 12-byte words).
#ifdef SPMV_ABLATIONS
// measurement build only: per workgroup of the last k_spmv_sweep_packed launch, the 100 MHz
// real-time clock at its start, at the end of its sweep and after its y / partial store, and its
// XCC and HW_ID registers (tools/wg_timeline.py reads them with spmv_abl_wg_times)
__device__ unsigned long long g_abl_wg[4 * 4096];
#define ABL_WG_STAMP(k)                                                                            \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                                 \
            g_abl_wg[4 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
#define ABL_WG_IDS()                                                                               \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                                 \
            g_abl_wg[4 * blockIdx.x + 3] = ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) | \
                                           (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    \
    } while (0)
#else
#define ABL_WG_STAMP(k) \
    do {                \
    } while (0)
#define ABL_WG_IDS() \
    do {             \
    } while (0)
#endif
// Work stealing among the pieces of a panel (split plans, ST; measurement build only, variants
// 37-39 -- it lost 3.5-5.5 % to the static split): a unit's workgroup iterations are
// tasks. Its first S = static_iters(n) tasks are its own (all but the last tail16/16 of them, at
// least kAhead); the rest it claims one at a time from the front of its counter (steal[u], low
// word), and once those are gone it claims iterations from the back of its sibling pieces (high
// word of theirs). Siblings share the panel, so a stolen iteration adds into the thief's own LDS
// rows and partial sums; k_sweep_combine adds every piece's partials as before and re-arms the
// counters. An owner's front claim of iteration S + f and a thief's back claim of n - 1 - b are
// granted only while S + f + b < n, read from the same 64-bit word by the same atomic add, so no
// iteration is taken twice or left out. The siblings' column ranges lie on other XCDs (pieces are
// dealt round-robin), so a stolen iteration gathers x lines its own L2 does not hold: stealing
// pays only in the tail.
struct SweepThief {
    uint32_t self, u0, pieces, k;  // own unit, first unit of the panel, pieces, siblings tried
    uint32_t vic, vn, vs;          // unit claimed from (self while front), its iterations, its static ones
    uint64_t ve0, ve1;             // its entry range
    uint32_t tail16;               // claimable share of a unit's iterations, in 16ths
    bool front, end;
};

// iterations a unit of n keeps without claiming: all but the last tail16/16, at least `ahead`
__device__ __forceinline__ uint32_t static_iters(uint32_t n, uint32_t tail16, uint32_t ahead)
{
    const uint32_t tail = (uint32_t)(((uint64_t)n * tail16 + 15) / 16);
    return n <= ahead ? n : (n - tail > ahead ? n - tail : ahead);
}

__device__ __forceinline__ unsigned long long thief_issue(const SweepThief &t, unsigned long long *steal)
{
    return __hip_atomic_fetch_add(steal + t.vic, t.front ? 1ull : (1ull << 32), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}

// the claim `old` (the counter before this add) granted: (b, e) = the task's entries
__device__ __forceinline__ bool thief_take(const SweepThief &t, unsigned long long old, uint32_t qg, uint32_t ahead,
                                           uint64_t &b, uint64_t &e)
{
    (void)ahead;
    const uint32_t f = (uint32_t)old, k = (uint32_t)(old >> 32);
    if ((uint64_t)t.vs + f + k >= t.vn)
        return false;
    const uint32_t it = t.front ? t.vs + f : t.vn - 1 - k;
    b = t.ve0 + (uint64_t)it * qg;
    e = t.ve1;
    return true;
}

// the next sibling piece (cyclic after this unit), or the end
__device__ __forceinline__ void thief_next(SweepThief &t, const uint32_t *__restrict__ unit_ent, uint32_t qg,
                                           uint32_t ahead)
{
    t.front = false;
    if (++t.k >= t.pieces) {
        t.end = true;
        return;
    }
    t.vic = t.u0 + (t.self - t.u0 + t.k) % t.pieces;
    t.ve0 = unit_ent[t.vic];
    t.ve1 = unit_ent[t.vic + 1];
    t.vn = (uint32_t)((t.ve1 - t.ve0 + qg - 1) / qg);
    t.vs = static_iters(t.vn, t.tail16, ahead);
}

// claims until a task is granted (true) or none is left anywhere (false)
__device__ bool thief_claim_sync(SweepThief &t, unsigned long long *steal, const uint32_t *__restrict__ unit_ent,
                                 uint32_t qg, uint32_t ahead, uint64_t &b, uint64_t &e)
{
    while (!t.end) {
        if (thief_take(t, thief_issue(t, steal), qg, ahead, b, e))
            return true;
        thief_next(t, unit_ent, qg, ahead);
    }
    return false;
}

// The combine of the PREVIOUS step run by extra workgroups of this step's sweep launch
// (spmv_plan_run_graph of a split plan, the "behind" form): blocks nunits.. of the grid are
// dispatched after every sweep unit, so they start on the CUs no unit holds and on those whose
// unit has finished (the sweep's tail). They claim chunks of kBehindRows rows of a panel from
// *ccount until none is left and add the pieces' partial sums in piece order, as
// k_sweep_combine does (the same y bit for bit). The previous step's partials (cpart) are not
// the ones this step's units write, and the rows they store are those of split panels, which the
// units leave to the partials. A chunk is J * T rows (J = 4 by default; the tools build's
// SPMV_BEHIND_ROWS measures others).
template <typename V, int T, typename A, uint32_t J>
__device__ void combine_behind(const uint32_t *__restrict__ panel_row, const uint32_t *__restrict__ panel_unit,
                               const A *__restrict__ cpart, uint32_t stride, V *__restrict__ y,
                               uint32_t *__restrict__ ccount, uint32_t npanels)
{
    constexpr uint32_t kBehindRows = J * T;
    const uint32_t cpp = (stride + kBehindRows - 1) / kBehindRows;  // chunks per panel
    __shared__ uint32_t claim;
    for (;;) {
        if (threadIdx.x == 0)
            claim = __hip_atomic_fetch_add(ccount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t c = claim;
        __syncthreads();
        if (c >= npanels * cpp)
            return;
        const uint32_t p = c / cpp, i0 = (c % cpp) * kBehindRows;
        const uint32_t u0 = panel_unit[p], pieces = panel_unit[p + 1] - u0;
        const uint32_t r0 = panel_row[p], R = panel_row[p + 1] - r0;
        if (pieces < 2 || i0 >= R)
            continue;
        const A *src = cpart + (uint64_t)u0 * stride;
        A acc[J];
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) {
            const uint32_t i = i0 + j * T + threadIdx.x;
            acc[j] = i < R ? src[i] : A(0);
        }
        for (uint32_t t = 1; t < pieces; ++t) {
            const A *sp = src + (uint64_t)t * stride;
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {
                const uint32_t i = i0 + j * T + threadIdx.x;
                acc[j] += i < R ? sp[i] : A(0);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) {
            const uint32_t i = i0 + j * T + threadIdx.x;
            if (i < R)
                y[r0 + i] = V(acc[j]);
        }
    }
}

// The packed sweep. FL... is empty for every launch but one: spmv_hw's streamed copy-back
// launches it with (uint32_t *yflag, uint32_t yepoch, V *yhost) -- each panel flagged in host
// memory once its y is stored (and, in the tools build's direct form, stored into host memory).
// With FL empty the kernel is the plain sweep, instruction for instruction the kernel before the
// flags existed (same registers, same 176-byte argument block) and as fast (418.6-420.3 vs
// 418.8-420.1 GFLOP/s, interleaved on one box); one kernel taking the extra arguments measured
// 1.3 % slower on the headline matrix, and so did a body shared by two entry points through a
// force-inlined function (profiles/r06u_flag_kernel_ab.txt).
template <typename V, int T, int Q, bool NT, int LAG = 0, int ABL = 0, typename A = double, bool DL = false,
          bool ST = false, typename... FL>
__global__ __launch_bounds__(T) void k_spmv_sweep_packed(
    const uint32_t *__restrict__ rc, const uint32_t *__restrict__ cbase, const V *__restrict__ val,
    const uint32_t *__restrict__ panel_row, const uint32_t *__restrict__ unit_ent,
    const uint32_t *__restrict__ unit_panel, const uint32_t *__restrict__ panel_unit,
    A *__restrict__ part, uint32_t stride, uint32_t *__restrict__ pcnt, const V *__restrict__ x,
    V *__restrict__ y, const uint16_t *__restrict__ row16, const uint8_t *__restrict__ d8,
    const uint32_t *__restrict__ dbase, const uint32_t *__restrict__ side, unsigned long long *__restrict__ steal,
    uint32_t tail16, uint32_t nunits, const A *__restrict__ cpart, uint32_t *__restrict__ ccount,
    uint32_t *__restrict__ cnext, uint32_t npanels, uint32_t cj, FL... fl)
{
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
    typedef uint8_t u8x2 __attribute__((ext_vector_type(2)));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    A *ylds = reinterpret_cast<A *>(smem);
    if (blockIdx.x >= nunits) {  // the previous step's combine, behind this step's units
        if (cj == 2)
            combine_behind<V, T, A, 2>(panel_row, panel_unit, cpart, stride, y, ccount, npanels);
        else if (cj == 8)
            combine_behind<V, T, A, 8>(panel_row, panel_unit, cpart, stride, y, ccount, npanels);
        else
            combine_behind<V, T, A, 4>(panel_row, panel_unit, cpart, stride, y, ccount, npanels);
        return;
    }
    if (cnext && blockIdx.x == 0 && threadIdx.x == 0)  // the next launch's claim counter
        __hip_atomic_store(cnext, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t p = unit_panel[blockIdx.x];  // unit = a piece of a panel's column-sorted entries
    const uint32_t pieces = panel_unit[p + 1] - panel_unit[p];
    const uint32_t r0 = panel_row[p], R = panel_row[p + 1] - r0;
    const uint64_t e0 = unit_ent[blockIdx.x], e1 = unit_ent[blockIdx.x + 1];
    __shared__ uint32_t progress[T / 64];
    constexpr uint64_t kGroup = 2ull * T;
    // ST: the ring of tasks (the entry range of one workgroup iteration) that thread 0 fills
    // kAhead tasks ahead of itself; the loose sync keeps every wave within LAG < kAhead tasks
    constexpr uint32_t QG = Q * (uint32_t)kGroup, kRing = 8, kAhead = 3;
    static_assert(!ST || (LAG > 0 && LAG < (int)kAhead && kAhead + LAG + 1 <= kRing), "steal ring sizing");
    __shared__ uint32_t ring_b[ST ? kRing : 1], ring_e[ST ? kRing : 1], ring_s[ST ? kRing : 1];
    SweepThief th{blockIdx.x, 0, pieces, 0, blockIdx.x, 0, 0, e0, e1, tail16, true, true};
    ABL_WG_STAMP(0);
    ABL_WG_IDS();
    for (uint32_t i = threadIdx.x; i <= R; i += T)
        ylds[i] = A(0);
    if (threadIdx.x < T / 64)
        progress[threadIdx.x] = 0;
    if constexpr (ST) {
        if (threadIdx.x == 0) {
            th.u0 = panel_unit[p];
            th.vn = (uint32_t)((e1 - e0 + QG - 1) / QG);
            th.vs = static_iters(th.vn, tail16, kAhead);
            th.end = false;
            for (uint32_t t = 0; t < kAhead; ++t) {  // the unit's first tasks are its own
                uint64_t b = 0, e = 0;
                bool got = t < th.vs;
                if (got)
                    b = e0 + (uint64_t)t * QG, e = e1;
                else
                    got = thief_claim_sync(th, steal, unit_ent, QG, kAhead, b, e);
                ring_b[t] = got ? (uint32_t)b : 0xFFFFFFFFu;
                ring_e[t] = got ? (uint32_t)e : 0u;
                ring_s[t] = t + 1;
            }
        }
    }
    __syncthreads();
    uint32_t iter = 0;
    A sink = 0;  // ablations 8/9 only
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane2 = 2u * (threadIdx.x & 63);
    uint64_t base = e0, bound = e1;  // this iteration's entries: [base, base + QG) below bound
    unsigned long long pend = 0;     // ST, thread 0: the claim issued for task s + kAhead
    bool issued = false;
    for (uint32_t s = 0;; ++s) {
        if constexpr (ST) {
            // task s + kAhead: one of the unit's static iterations, or a claim issued here whose
            // result is consumed after this task's gathers
            issued = false;
            if (threadIdx.x == 0 && !th.end && !(th.front && s + kAhead < th.vs)) {
                pend = thief_issue(th, steal);
                issued = true;
            }
            const uint32_t slot = s % kRing;
            // written kAhead tasks ago unless thread 0 is in a claim loop (the tail); bounded wait
            uint32_t spin = 0;
            while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ring_s[slot], __ATOMIC_ACQUIRE,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP)) != s + 1 &&
                   ++spin < (1u << 24))
                __builtin_amdgcn_s_sleep(1);
            const uint32_t rb = __builtin_amdgcn_readfirstlane(ring_b[slot]);
            if (rb == 0xFFFFFFFFu || spin >= (1u << 24))
                break;
            base = rb;
            bound = __builtin_amdgcn_readfirstlane(ring_e[slot]);
        } else {
            if (base >= e1)
                break;
        }
        // branch-free body: a group past the unit's end re-reads its last chunk (valid memory)
        // and adds into the scratch slot R, so every load of the Q groups issues together
        const uint64_t last_chunk = bound > e0 || ST ? bound - 128 : e0;
        u32x2 w[Q];
        uint32_t cb[Q];
        V v[Q][2];
        bool ok[Q];
        u16x2 r16[Q];  // DL only
        u8x2 dd[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            uint64_t wbase = base + q * kGroup + 128ull * wave;  // this wave's chunk
            ok[q] = wbase < bound;                                // wave-uniform
            wbase = ok[q] ? wbase : last_chunk;
            if constexpr (ABL == 3 || ABL == 4 || ABL == 9)  // ablation: entries re-read from the unit's first 4K (L2-resident)
                wbase = e0 + ((wbase - e0) & 4095u);
            const uint64_t e = wbase + lane2;
            if constexpr (DL) {
                r16[q] = lds_<NT>(reinterpret_cast<const u16x2 *>(row16 + e));
                dd[q] = lds_<NT>(reinterpret_cast<const u8x2 *>(d8 + e));
                cb[q] = dbase[wbase >> 7];
                loadv<NT, 2>(val, e, v[q]);
                continue;
            }
            if constexpr (ABL == 11) {
                // ablation (wrong y): an 11-byte entry stream -- u16 row + u8 column delta per
                // entry from two regions of the rc array (2 + 1 B instead of 4), columns decoded by
                // a 64-lane prefix sum of the deltas (the cost of delta-coded columns)
                typedef uint16_t u16x2_t __attribute__((ext_vector_type(2)));
                typedef uint8_t u8x2_t __attribute__((ext_vector_type(2)));
                const u16x2_t r16 = lds_<NT>(reinterpret_cast<const u16x2_t *>(reinterpret_cast<const uint16_t *>(rc) + e));
                const u8x2_t d8 = lds_<NT>(reinterpret_cast<const u8x2_t *>(
                    reinterpret_cast<const uint8_t *>(rc) + 2 * (uint64_t)unit_ent[gridDim.x] + e));
                const uint32_t dsum = (uint32_t)(d8.x & 63u) + (uint32_t)(d8.y & 63u);
                // 64-lane inclusive prefix sum by DPP (the binned kernel's row-delta decode)
                uint32_t inc = dsum;
                inc += __builtin_amdgcn_update_dpp(0u, dsum, 0x111, 0xf, 0xf, true);
                inc += __builtin_amdgcn_update_dpp(0u, dsum, 0x112, 0xf, 0xf, true);
                inc += __builtin_amdgcn_update_dpp(0u, dsum, 0x113, 0xf, 0xf, true);
                inc += __builtin_amdgcn_update_dpp(0u, inc, 0x114, 0xf, 0xe, true);
                inc += __builtin_amdgcn_update_dpp(0u, inc, 0x118, 0xf, 0xc, true);
                inc += __builtin_amdgcn_update_dpp(0u, inc, 0x142, 0xa, 0xf, false);
                inc += __builtin_amdgcn_update_dpp(0u, inc, 0x143, 0xc, 0xf, false);
                const uint32_t c0 = inc - dsum + (d8.x & 63u);
                w[q].x = ((uint32_t)(r16.x & 16383u) << 16) | (c0 & 0xFFFFu);
                w[q].y = ((uint32_t)(r16.y & 16383u) << 16) | ((c0 + (d8.y & 63u)) & 0xFFFFu);
            } else {
                w[q] = lds_<NT>(reinterpret_cast<const u32x2 *>(rc + e));
            }
            cb[q] = cbase[wbase >> 7];
            if constexpr (ABL == 10) {  // ablation: one value per two entries (8 B/entry streamed, not 12)
                v[q][0] = v[q][1] = lds_<NT>(val + (wbase >> 1) + (lane2 >> 1));
            } else {
                loadv<NT, 2>(val, e, v[q]);
            }
        }
        V xv[Q][2];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            // ABL (measurement-only ablations, variants 60/61): 1 = x index folded into a 256 KiB
            // window (every gather an L2 hit, same request count), 2 = no gathers
            if constexpr (DL) {
                // per group: its columns, then its two gathers (decoding every group's columns
                // before any gather measured 3 % slower, profiles/r03_delta_columns.jsonl)
                uint32_t cx, cy;
                if (cb[q] & 0x80000000u) {  // wave-uniform: a chunk with a gap > 511
                    const uint64_t sb = (uint64_t)(cb[q] & 0x7FFFFFFFu) * kSweepChunk + lane2;
                    const u32x2 cc = lds_<NT>(reinterpret_cast<const u32x2 *>(side + sb));
                    cx = cc.x;
                    cy = cc.y;
                } else {
                    // 9-bit deltas: bit 15 of the row word is the delta's bit 8 (rows < 32768)
                    const uint32_t dx = dd[q].x | ((uint32_t)(r16[q].x >> 15) << 8);
                    const uint32_t dy = dd[q].y | ((uint32_t)(r16[q].y >> 15) << 8);
                    const uint32_t i0 = wave_inclusive_sum(dx), i1 = wave_inclusive_sum(dy);
                    cx = cb[q] + i0;
                    cy = cb[q] + (uint32_t)__builtin_amdgcn_readlane(i0, 63) + i1;
                }
                xv[q][0] = x[cx];
                xv[q][1] = x[cy];
            } else if constexpr (ABL == 2 || ABL == 5) {
                xv[q][0] = V(w[q].x & 1u);
                xv[q][1] = V(w[q].y & 1u);
            } else if constexpr (ABL == 6) {  // x gathers non-temporal (nt)
                xv[q][0] = __builtin_nontemporal_load(x + cb[q] + (w[q].x & 0xFFFFu));
                xv[q][1] = __builtin_nontemporal_load(x + cb[q] + (w[q].y & 0xFFFFu));
            } else if constexpr (ABL == 7) {  // x gathers L1-bypassing (sc1)
                xv[q][0] = __hip_atomic_load(x + cb[q] + (w[q].x & 0xFFFFu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                xv[q][1] = __hip_atomic_load(x + cb[q] + (w[q].y & 0xFFFFu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const uint32_t m = (ABL == 1 || ABL == 4 || ABL == 9) ? 0x7FFFu : 0xFFFFFFFFu;
                xv[q][0] = x[(cb[q] + (w[q].x & 0xFFFFu)) & m];
                xv[q][1] = x[(cb[q] + (w[q].y & 0xFFFFu)) & m];
            }
        }
        if constexpr (ABL == 8 || ABL == 9) {  // ablation: no LDS adds (register sum)
#pragma unroll
            for (int q = 0; q < Q; ++q)
                sink += A(v[q][0]) * A(xv[q][0]) + A(v[q][1]) * A(xv[q][1]);
        } else {
            uint32_t ri[2 * Q];
            A pv[2 * Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                if constexpr (DL) {
                    ri[2 * q] = ok[q] ? (uint32_t)(r16[q].x & 0x7FFFu) : R;
                    ri[2 * q + 1] = ok[q] ? (uint32_t)(r16[q].y & 0x7FFFu) : R;
                } else {
                    ri[2 * q] = ok[q] ? (w[q].x >> 16) : R;
                    ri[2 * q + 1] = ok[q] ? (w[q].y >> 16) : R;
                }
                pv[2 * q] = A(v[q][0]) * A(xv[q][0]);
                pv[2 * q + 1] = A(v[q][1]) * A(xv[q][1]);
            }
            lds_add_n<2 * Q>(ylds, ri, pv);
        }
        if constexpr (ST) {
            if (threadIdx.x == 0) {  // the task kAhead ahead: the claim issued above, or a claim loop
                uint64_t b = 0, e = 0;
                bool got = false;
                if (issued) {
                    got = thief_take(th, pend, QG, kAhead, b, e);
                    if (!got) {
                        thief_next(th, unit_ent, QG, kAhead);
                        got = thief_claim_sync(th, steal, unit_ent, QG, kAhead, b, e);
                    }
                } else if (!th.end && th.front && s + kAhead < th.vs) {
                    got = true;
                    b = e0 + (uint64_t)(s + kAhead) * QG;
                    e = e1;
                }
                const uint32_t slot = (s + kAhead) % kRing;
                ring_b[slot] = got ? (uint32_t)b : 0xFFFFFFFFu;
                ring_e[slot] = got ? (uint32_t)e : 0u;
                __hip_atomic_store(&ring_s[slot], s + kAhead + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            base += QG;
        }
        if constexpr (LAG == 0) {
            __syncthreads();
        } else {
            ++iter;
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store(&progress[wave], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // wait while more than LAG iterations ahead of the slowest wave
            for (;;) {
                const uint32_t lane = threadIdx.x & 63;
                uint32_t pr = lane < T / 64
                                  ? __hip_atomic_load(&progress[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                                  : 0xFFFFFFFFu;
#pragma unroll
                for (int d = 1; d < T / 64; d <<= 1) {
                    const uint32_t o = __shfl_xor(pr, d, 64);
                    pr = o < pr ? o : pr;
                }
                if (__builtin_amdgcn_readfirstlane(pr) + LAG >= iter)
                    break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    if constexpr (ABL == 8 || ABL == 9)
        lds_add(&ylds[R], sink);
    __syncthreads();
    ABL_WG_STAMP(1);
    if constexpr (sizeof...(FL) == 0) {
        write_panel<V, T, A>(ylds, R, y + r0, pieces, part, stride, panel_unit[p], pcnt ? pcnt + p : nullptr);
    } else {
        // spmv_hw's streamed copy-back (plans of one piece per panel only). yhost: the tools
        // build's direct form -- the panel's y stored straight into pinned host memory over PCIe
        // instead of device memory. Then the panel's y is published at system scope -- every
        // wave's stores complete, one lane's release writes the XCD L2's dirty lines back to
        // memory -- and its flag in host memory is set to this call's epoch; the host copies the
        // panel's rows while the other panels still sweep
        const auto args = std::make_tuple(fl...);
        uint32_t *yflag = std::get<0>(args);
        const uint32_t yepoch = std::get<1>(args);
        V *yhost = std::get<2>(args);
        write_panel<V, T, A>(ylds, R, (yhost ? yhost : y) + r0, pieces, part, stride, panel_unit[p],
                             pcnt ? pcnt + p : nullptr);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(yflag + p, yepoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ABL_WG_STAMP(2);
}


// Deterministic form (env SPMV_SWEEP_DETERMINISTIC=1): the same plan, layout and gathers as
// k_spmv_sweep_packed / k_spmv_sweep, but the LDS adds of a workgroup are ordered. In the default
// kernels all 16 waves add into any row of the panel in timing order, so y changes in its last
// bits from run to run. Here an LDS token `turn` passes from wave to wave: wave w adds the
// products of its iteration i only when turn == i * W + w, then hands the token on. Every row
// therefore receives its products in the order (iteration, wave, lane) that the plan alone
// defines, and y is bitwise the same on every run and for every plan built from the same CSR --
// the fixed-order accumulation of compute_results (spmv.cpp:66-104), in an order of its own --
// while each gather instruction still covers 64 consecutive column-sorted entries of the whole
// panel (the x-line sharing of the default form).
// The token serialises only the short add phases. Each step i issues the gathers of i + 2 and
// the entry loads of i + 4 before it waits for the token, so two iterations of gathers stay in
// flight while the waves take turns (the loop body is unrolled 6 times -- 2 entry buffers x 3
// gathered buffers -- so that no register with a load in flight is ever copied).
// ORD = 0 (default): the wave's adds complete (lgkmcnt 0) before a release store of the token,
// and the next wave acquires it before its adds: the order follows from the memory model alone
// (3 % slower than ORD 1, profiles/r02_ab_variants.jsonl r02w). ORD = 1 (variant 91, kept for
// measurements): the token store follows the adds' issue (compiler ordering only), which is
// correct only if the LDS executes a CU's requests in arrival order -- observed, not documented.
// PK: packed 12-byte entries (rc + chunk base); otherwise the 14-byte form (s_col, s_row).
template <typename V, int T, int Q, bool PK, int ORD, typename A = double>
__global__ __launch_bounds__(T) void k_spmv_sweep_turn(
    const uint32_t *__restrict__ col, const uint32_t *__restrict__ cbase, const uint16_t *__restrict__ srow16,
    const V *__restrict__ val, const uint32_t *__restrict__ panel_row, const uint32_t *__restrict__ unit_ent,
    const uint32_t *__restrict__ unit_panel, const uint32_t *__restrict__ panel_unit, A *__restrict__ part,
    uint32_t stride, uint32_t *__restrict__ pcnt, const V *__restrict__ x, V *__restrict__ y)
{
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t W = T / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    A *ylds = reinterpret_cast<A *>(smem);
    __shared__ uint32_t turn;
    __shared__ uint32_t progress[W];  // ORD 2 only
    const uint32_t p = unit_panel[blockIdx.x];
    const uint32_t pieces = panel_unit[p + 1] - panel_unit[p];
    const uint32_t r0 = panel_row[p], R = panel_row[p + 1] - r0;
    const uint64_t e0 = unit_ent[blockIdx.x], e1 = unit_ent[blockIdx.x + 1];
    for (uint32_t i = threadIdx.x; i <= R; i += T)
        ylds[i] = A(0);
    if (threadIdx.x == 0)
        turn = 0;
    if (threadIdx.x < W)
        progress[threadIdx.x] = 0;
    __syncthreads();
    constexpr uint64_t kGroup = 2ull * T;
    constexpr uint64_t kStep = Q * kGroup;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane2 = 2u * (threadIdx.x & 63);
    const uint64_t last_chunk = e1 > e0 ? e1 - 128 : e0;
    struct EB {  // entries of one iteration
        u32x2 w[Q];      // packed rc words, or absolute columns
        uint32_t cb[Q];  // chunk bases (packed form)
        u16x2 r[Q];      // rows in the panel (14-byte form)
        V v[Q][2];
        bool ok[Q];
    };
    struct DB {  // gathered x, values and LDS slots of one iteration
        V x[Q][2], v[Q][2];
        uint32_t r[2 * Q];
    };
    auto ld = [&](uint64_t base, EB &e) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            uint64_t wbase = base + q * kGroup + 128ull * wave;
            e.ok[q] = wbase < e1;  // wave-uniform; a group past the end re-reads the last chunk
            wbase = e.ok[q] ? wbase : last_chunk;
            const uint64_t ei = wbase + lane2;
            e.w[q] = lds_<true>(reinterpret_cast<const u32x2 *>(col + ei));
            if constexpr (PK)
                e.cb[q] = cbase[wbase >> 7];
            else
                e.r[q] = lds_<true>(reinterpret_cast<const u16x2 *>(srow16 + ei));
            loadv<true, 2>(val, ei, e.v[q]);
        }
    };
    auto gat = [&](const EB &e, DB &d) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if constexpr (PK) {
                d.x[q][0] = x[e.cb[q] + (e.w[q].x & 0xFFFFu)];
                d.x[q][1] = x[e.cb[q] + (e.w[q].y & 0xFFFFu)];
                d.r[2 * q] = e.ok[q] ? (e.w[q].x >> 16) : R;
                d.r[2 * q + 1] = e.ok[q] ? (e.w[q].y >> 16) : R;
            } else {
                d.x[q][0] = x[e.w[q].x];
                d.x[q][1] = x[e.w[q].y];
                d.r[2 * q] = e.ok[q] ? (uint32_t)e.r[q].x : R;
                d.r[2 * q + 1] = e.ok[q] ? (uint32_t)e.r[q].y : R;
            }
            d.v[q][0] = e.v[q][0];
            d.v[q][1] = e.v[q][1];
        }
    };
    auto step = [&](uint64_t base, uint32_t my, EB &e, const DB &cur, DB &fill) {
        gat(e, fill);             // gathers of i + 2
        ld(base + 4 * kStep, e);  // entries of i + 4 (past the end: the last chunk, unused)
        A pv[2 * Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            pv[2 * q] = A(cur.v[q][0]) * A(cur.x[q][0]);
            pv[2 * q + 1] = A(cur.v[q][1]) * A(cur.x[q][1]);
        }
        if constexpr (ORD >= 2) {  // measurement only: unordered adds (2: waves at most 2 steps apart)
            lds_add_n<2 * Q>(ylds, cur.r, pv);
            if constexpr (ORD == 2) {
                const uint32_t iter = my / W + 1;
                if ((threadIdx.x & 63) == 0)
                    __hip_atomic_store(&progress[wave], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                for (;;) {
                    const uint32_t lane = threadIdx.x & 63;
                    uint32_t pr = lane < W ? __hip_atomic_load(&progress[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                                           : 0xFFFFFFFFu;
#pragma unroll
                    for (int d = 1; d < (int)W; d <<= 1) {
                        const uint32_t o = __shfl_xor(pr, d, 64);
                        pr = o < pr ? o : pr;
                    }
                    if (__builtin_amdgcn_readfirstlane(pr) + 2 >= iter)
                        break;
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            return;
        }
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&turn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != my) {
        }
        lds_add_n<2 * Q>(ylds, cur.r, pv);
        if constexpr (ORD == 0) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's adds are done
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store(&turn, my + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // compiler order only: adds, then the store
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store(&turn, my + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    // 32-bit scalar trip count: all waves of the workgroup take the same number of steps. An
    // empty unit (no entries at all: the prologue's loads would read past a 4-entry allocation)
    // only writes its zeros.
    const uint32_t nit = (uint32_t)((e1 - e0 + kStep - 1) / kStep);
    if (nit == 0) {
        __syncthreads();
        write_panel<V, T, A>(ylds, R, y + r0, pieces, part, stride, panel_unit[p], pcnt ? pcnt + p : nullptr);
        return;
    }
    EB ea, eb;
    DB d0, d1, d2;
    ld(e0, ea);
    ld(e0 + kStep, eb);
    gat(ea, d0);
    ld(e0 + 2 * kStep, ea);
    gat(eb, d1);
    ld(e0 + 3 * kStep, eb);
    uint32_t my = wave;
    uint64_t base = e0;
    uint32_t it = 0;
#define TSTEP(E, C, F)       \
    step(base, my, E, C, F); \
    base += kStep;           \
    my += W;                 \
    if (++it >= nit)         \
        break;
    while (it < nit) {
        TSTEP(ea, d0, d2)
        TSTEP(eb, d1, d0)
        TSTEP(ea, d2, d1)
        TSTEP(eb, d0, d2)
        TSTEP(ea, d1, d0)
        TSTEP(eb, d2, d1)
    }
#undef TSTEP
    if constexpr (ORD == 2)  // a finished wave never holds the others back
        if ((threadIdx.x & 63) == 0)
            __hip_atomic_store(&progress[wave], 0xFFFFFFF0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    write_panel<V, T, A>(ylds, R, y + r0, pieces, part, stride, panel_unit[p], pcnt ? pcnt + p : nullptr);
}

// group c of G entries (a 128-entry chunk): base = min column; fails the plan's packing when the
// span >= 65536
__global__ void k_sweep_chunk_base(const uint32_t *__restrict__ col, uint64_t nchunks, uint32_t G,
                                   uint32_t *__restrict__ cbase, uint32_t *__restrict__ bad, uint8_t *__restrict__ wide)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks)
        return;
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t k = 0; k < G; ++k) {
        const uint32_t v = col[c * G + k];
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    cbase[c] = lo;
    wide[c] = hi - lo >= 65536u;
    if (hi - lo >= 65536u)
        atomicAdd(bad, 1u);  // (the number of wide chunks)
}

// in place: col[k] <- (row << 16) | (col - base of k's group of 2^gshift entries); a wide group
// (its columns span >= 65536) keeps offset 0 here -- its absolute columns go to the side table
__global__ void k_sweep_pack_rc(uint32_t *__restrict__ col, const uint16_t *__restrict__ row,
                                const uint32_t *__restrict__ cbase, uint64_t n, uint32_t gshift,
                                const uint8_t *__restrict__ wide)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint64_t c = k >> gshift;
    col[k] = ((uint32_t)row[k] << 16) | (wide[c] ? 0u : col[k] - cbase[c]);
}

// the lane-order permutation of k_sweep_lane_order applied to one u32 array (a wide plan's
// absolute columns, which follow their entries into the side table)
__global__ void k_sweep_lane_order_u32(const uint32_t *__restrict__ in, uint64_t n, uint32_t *__restrict__ out)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint64_t c = k & ~(uint64_t)127, w = k & 127;
    out[c + 2 * (w & 63) + (w >> 6)] = in[k];
}

// Lane-order permutation inside each 128-entry chunk: memory word 2l+j holds logical entry
// 64j+l, so the j-th gather instruction of a wave covers 64 CONSECUTIVE entries (sorted by
// column) and lanes whose columns share a 128-byte x line are served by one L2 request.
template <typename V>
__global__ void k_sweep_lane_order(const uint32_t *__restrict__ rc_in, const V *__restrict__ v_in, uint64_t n,
                                   uint32_t *__restrict__ rc_out, V *__restrict__ v_out)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint64_t c = k & ~(uint64_t)127, w = k & 127;
    const uint64_t m = c + 2 * (w & 63) + (w >> 6);
    rc_out[m] = rc_in[k];
    v_out[m] = v_in[k];
}

// Delta-coded columns of a lane-ordered packed chunk (one thread per chunk). The chunk's entries
// are first put in ascending column order (the radix sort keys drop the low `shift` column bits
// for large matrices, so entries of one bucket keep their CSR order; rc words and values move
// together, in place). Then per entry: the column minus the previous column of the same wave
// instruction (the first of instruction 0 from the chunk base; instruction 1 continues from entry
// 63) as 9 bits -- the low 8 in d8, bit 8 in bit 15 of the row word (panel rows < 32768) -- and
// the row, in lane order; flag = some gap > 511 (the chunk's columns go to the side table).
template <typename V>
__global__ void k_sweep_delta(uint32_t *__restrict__ rc, V *__restrict__ val, uint64_t nchunks,
                              uint16_t *__restrict__ row16, uint8_t *__restrict__ d8, uint8_t *__restrict__ flag,
                              const uint8_t *__restrict__ wide)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks)
        return;
    constexpr int G = (int)kSweepChunk;
    uint32_t w[G];
    V v[G];
    uint32_t *cw = rc + c * G;
    V *cv = val + c * G;
    for (int k = 0; k < G; ++k) {  // logical entry k sits at word 2 (k mod 64) + k / 64
        const int m = 2 * (k & 63) + (k >> 6);
        w[k] = cw[m];
        v[k] = cv[m];
    }
    for (int k = 1; k < G; ++k) {  // stable insertion sort by column offset (nearly sorted input)
        const uint32_t wk = w[k];
        const V vk = v[k];
        int j = k - 1;
        while (j >= 0 && (w[j] & 0xFFFFu) > (wk & 0xFFFFu)) {
            w[j + 1] = w[j];
            v[j + 1] = v[j];
            --j;
        }
        w[j + 1] = wk;
        v[j + 1] = vk;
    }
    uint32_t prev = 0;
    bool big = false;
    for (int k = 0; k < G; ++k) {
        const int m = 2 * (k & 63) + (k >> 6);
        const uint32_t off = w[k] & 0xFFFFu;
        const uint32_t d = off - prev;
        big |= d > 511u;
        cw[m] = w[k];
        cv[m] = v[k];
        row16[c * G + m] = (uint16_t)((w[k] >> 16) | ((d >> 8) & 1u) << 15);
        d8[c * G + m] = (uint8_t)d;
        prev = off;
    }
    flag[c] = big || wide[c] ? 1 : 0;  // (a wide chunk's offsets are all 0: the sort kept its order)
}

// per chunk: dbase = the chunk base, or bit 31 | its side-table index (sidx[c] != ~0), whose 128
// absolute columns are written in lane order
__global__ void k_sweep_delta_base(const uint32_t *__restrict__ rc, const uint32_t *__restrict__ cbase,
                                   const uint32_t *__restrict__ sidx, uint64_t nchunks, uint32_t *__restrict__ dbase,
                                   uint32_t *__restrict__ side, const uint8_t *__restrict__ wide,
                                   const uint32_t *__restrict__ abs_col)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks)
        return;
    const uint32_t k = sidx[c];
    if (k == 0xFFFFFFFFu) {
        dbase[c] = cbase[c];
        return;
    }
    dbase[c] = 0x80000000u | k;
    for (uint64_t m = 0; m < kSweepChunk; ++m)  // (wide: the lane-ordered absolute columns)
        side[(uint64_t)k * kSweepChunk + m] =
            wide[c] ? abs_col[c * kSweepChunk + m] : cbase[c] + (rc[c * kSweepChunk + m] & 0xFFFFu);
}

// the 12-byte rc words of a delta plan, rebuilt from the delta arrays (one thread per chunk):
// column offsets are the running sums of the 9-bit deltas in logical entry order, or side-table
// columns minus the chunk base
__global__ void k_sweep_delta_decode(const uint16_t *__restrict__ row16, const uint8_t *__restrict__ d8,
                                     const uint32_t *__restrict__ dbase, const uint32_t *__restrict__ cbase,
                                     const uint32_t *__restrict__ side, uint64_t nchunks, uint32_t *__restrict__ rc)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks)
        return;
    constexpr int G = (int)kSweepChunk;
    const uint32_t db = dbase[c];
    uint32_t off = 0;
    for (int k = 0; k < G; ++k) {
        const uint64_t m = c * G + 2 * (k & 63) + (k >> 6);
        const uint32_t rw = row16[m];
        if (db & 0x80000000u)
            off = side[(uint64_t)(db & 0x7FFFFFFFu) * G + (m - c * G)] - cbase[c];
        else
            off += (uint32_t)d8[m] | ((rw >> 15) << 8);
        rc[m] = ((rw & 0x7FFFu) << 16) | off;
    }
}

// A delta plan keeps only the 11-byte entries; a kernel that reads the 12-byte rc words (the
// deterministic variants 91 / 94, variant 35, the ablations) gets them rebuilt here, once
int sweep_materialize_rc(spmv_plan &p)
{
    if (!p.sweep_delta || p.d_s_col || p.ent_pad == 0)
        return 0;
    if (p.sweep_wide) {  // chunks spanning >= 65536 columns have no 16-bit offsets
        set_error("sweep variant needs the 12-byte entries, which this plan's wide chunks cannot hold");
        return 1;
    }
    const uint64_t nchunks = p.ent_pad / kSweepChunk;
    SPMV_TRY(hipSetDevice(p.device));
    SPMV_TRY(hipMalloc((void **)&p.d_s_col, p.ent_pad * 4));
    hipLaunchKernelGGL(k_sweep_delta_decode, dim3((unsigned)((nchunks + 63) / 64)), dim3(64), 0, nullptr, p.d_s_row16,
                       p.d_s_d8, p.d_s_dbase, p.d_s_cbase, p.d_s_side, nchunks, p.d_s_col);
    SPMV_TRY(hipGetLastError());
    SPMV_TRY(hipDeviceSynchronize());
    return 0;
}

// sort key of every entry: (panel, column bucket); one thread per row
__global__ void k_sweep_keys(const IndexType *__restrict__ rp, const IndexType *__restrict__ col,
                             const uint32_t *__restrict__ panel_row, uint32_t npanels, IndexType nrows,
                             uint64_t nbuckets, uint32_t shift, uint32_t *__restrict__ keys,
                             uint32_t *__restrict__ idx)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows)
        return;
    // panel of row r: last p with panel_row[p] <= r
    uint32_t lo = 0, hi = npanels;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (panel_row[mid] <= r)
            lo = mid;
        else
            hi = mid;
    }
    const uint64_t pbase = (uint64_t)lo * nbuckets;
    for (IndexType j = rp[r]; j < rp[r + 1]; ++j) {
        keys[j] = (uint32_t)(pbase + (col[j] >> shift));
        idx[j] = j;
    }
}

// sorted position k -> padded position; carries column, in-panel row, value
template <typename V>
__global__ void k_sweep_scatter(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ idx,
                                uint64_t nnz, uint64_t nbuckets, const IndexType *__restrict__ rp,
                                IndexType nrows, const IndexType *__restrict__ col_src,
                                const V *__restrict__ val_src, const uint32_t *__restrict__ panel_row,
                                const uint32_t *__restrict__ off, const uint32_t *__restrict__ poff,
                                uint32_t *__restrict__ s_col, uint16_t *__restrict__ s_row,
                                V *__restrict__ s_val)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz)
        return;
    const uint32_t p = (uint32_t)(keys[k] / nbuckets);
    const uint32_t j = idx[k];
    // row of entry j: last r with rp[r] <= j (rows with entries only)
    uint32_t lo = 0, hi = nrows;
    while (hi - lo > 1) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (rp[mid] <= j)
            lo = mid;
        else
            hi = mid;
    }
    const uint64_t dst = (uint64_t)poff[p] + (k - off[p]);
    s_col[dst] = col_src[j];
    s_row[dst] = (uint16_t)(lo - panel_row[p]);
    s_val[dst] = val_src[j];
}

template <typename V>
__global__ void k_sweep_pad(uint32_t npanels, const uint32_t *__restrict__ panel_row,
                            const uint32_t *__restrict__ off, const uint32_t *__restrict__ poff,
                            uint32_t *__restrict__ s_col, uint16_t *__restrict__ s_row, V *__restrict__ s_val)
{
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npanels)
        return;
    const uint32_t R = panel_row[p + 1] - panel_row[p];
    const uint64_t first_pad = (uint64_t)poff[p] + (off[p + 1] - off[p]);
    const uint32_t pad_col = first_pad > poff[p] ? s_col[first_pad - 1] : 0u;
    for (uint64_t d = first_pad; d < poff[p + 1]; ++d) {
        s_col[d] = pad_col;  // value 0: adds nothing; column kept near the panel's last one
        s_row[d] = (uint16_t)R;  // scratch slot, never written back
        s_val[d] = V(0);
    }
}

// locality probe: fraction of sampled rows whose first two columns are < 64 apart
// Locality probe for the automatic kernel choice: over sampled rows, the fraction of
// consecutive column pairs (up to 64 per row) that lie < 64 columns apart. Random columns give
// ~0, a band 1, 2-D / 3-D stencils 0.3-0.7 (one jump per grid line or plane).
__global__ void k_locality(const IndexType *__restrict__ rp, const IndexType *__restrict__ col, IndexType nrows,
                           uint32_t stride, unsigned long long *__restrict__ counts)
{
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * stride;
    if (r >= nrows)
        return;
    const IndexType b = rp[r], e = rp[r + 1];
    if (e - b < 2)
        return;
    const IndexType last = e - b > 65 ? b + 65 : e;
    unsigned long long pairs = 0, near = 0;
    for (IndexType k = b + 1; k < last; ++k) {
        const IndexType c0 = col[k - 1], c1 = col[k];
        const IndexType d = c1 > c0 ? c1 - c0 : c0 - c1;
        ++pairs;
        near += d < 64;
    }
    atomicAdd(&counts[0], pairs);
    atomicAdd(&counts[1], near);
}

template <int T, typename A>
static void launch_sweep_t(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm,
                           void *part_buf, const sweep_behind &bh)
{
    const size_t lds = (size_t(p.panel_rmax) + 1) * sizeof(A);
    const dim3 grid((unsigned)p.nunits), block(T);
    const dim3 gridb((unsigned)p.nunits + (bh.cpart ? bh.blocks : 0u));  // + the combine behind
    A *part = reinterpret_cast<A *>(part_buf);
    uint32_t *pcnt = p.sweep_split > 1 && p.d_panel_cnt ? p.d_panel_cnt : nullptr;  // fused combine
    // Unpacked (14-B entries, used when a chunk spans >= 65536 columns): E entries per thread,
    // Q groups per barrier, SYNC barrier, NT non-temporal entry loads.
#define SWEEP(E, Q, SYNC, NT)                                                                     \
    launch_or_warm(warm, k_spmv_sweep<ValueType, T, E, Q, SYNC, NT, A>, grid, block, lds, s, p.d_s_col,   \
                       p.d_s_row, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, part, p.panel_rmax + 1, pcnt, d_x, d_y)
    // deterministic form (env SPMV_SWEEP_DETERMINISTIC=1, or variants 91 / 94 on any sweep plan)
#define TURN(PK, ORD)                                                                              \
    launch_or_warm(warm, k_spmv_sweep_turn<ValueType, T, 2, PK, ORD, A>, grid, block, lds, s, p.d_s_col,          \
                   p.d_s_cbase, p.d_s_row, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, \
                   part, p.panel_rmax + 1, pcnt, d_x, d_y)
#ifdef SPMV_ABLATIONS
    // measurement only: the turn kernel's pipeline without the ordering (52: loose sync, 51: none)
    if (p.sweep_packed && p.sweep_variant == 52) {
        TURN(true, 2);
        return;
    }
    if (p.sweep_packed && p.sweep_variant == 51) {
        TURN(true, 3);
        return;
    }
#endif
    if (p.sweep_det || p.sweep_variant == kSweepTurn || p.sweep_variant == kSweepTurnOrdered) {
        // ORD 0 (each wave's adds complete before the release hand-over) is the default of
        // SPMV_SWEEP_DETERMINISTIC=1: its ordering follows from the memory model alone. Variant 91
        // (tools library) keeps the 3 % faster ORD 1 hand-over (compiler ordering; relies on the
        // LDS executing a CU's requests in arrival order) for measurements.
#ifdef SPMV_ABLATIONS
        if (p.sweep_variant == kSweepTurn) {
            if (p.sweep_packed) TURN(true, 1); else TURN(false, 1);
            return;
        }
#endif
        if (p.sweep_packed) TURN(true, 0); else TURN(false, 0);
        return;
    }
#undef TURN
    if (p.sweep_packed) {
#define PKN(NT, Q, LAG, ABL)                                                                        \
    launch_or_warm(warm, k_spmv_sweep_packed<ValueType, T, Q, NT, LAG, ABL, A>, grid, block, lds, s, p.d_s_col, \
                       p.d_s_cbase, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, part, p.panel_rmax + 1, pcnt, d_x, d_y, \
                       (const uint16_t *)nullptr, (const uint8_t *)nullptr, (const uint32_t *)nullptr, (const uint32_t *)nullptr, \
                       (unsigned long long *)nullptr, 0u, (uint32_t)p.nunits, (const A *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, 0u)
    // the default kernel on delta-coded columns (variant 28's loose sync: 2 groups, lag 2)
#define PKD(ST, TAIL)                                                                                 \
    launch_or_warm(warm, k_spmv_sweep_packed<ValueType, T, 2, true, 2, 0, A, true, ST>, gridb, block, lds, s, p.d_s_col, \
                       p.d_s_cbase, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, part, p.panel_rmax + 1, pcnt, d_x, d_y, \
                       p.d_s_row16, p.d_s_d8, p.d_s_dbase, p.d_s_side, ST ? p.d_steal : (unsigned long long *)nullptr, (uint32_t)(TAIL), \
                       (uint32_t)p.nunits, reinterpret_cast<const A *>(bh.cpart), bh.ccount, bh.cnext, (uint32_t)p.npanels, bh.rows_per_thread)
    // spmv_hw's streamed copy-back (p.y_flag set: plans of one piece per panel, default variant)
#define PKDF()                                                                                        \
    launch_or_warm(warm, k_spmv_sweep_packed<ValueType, T, 2, true, 2, 0, A, true, false, uint32_t *, uint32_t, ValueType *>, gridb, block, lds, s, \
                   p.d_s_col, p.d_s_cbase, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, part, \
                   p.panel_rmax + 1, pcnt, d_x, d_y, p.d_s_row16, p.d_s_d8, p.d_s_dbase, p.d_s_side,               \
                   (unsigned long long *)nullptr, 0u, (uint32_t)p.nunits, (const A *)nullptr, (uint32_t *)nullptr,  \
                   (uint32_t *)nullptr, (uint32_t)p.npanels, 0u, p.y_flag, p.y_epoch, p.y_host)
#define PKF()                                                                                         \
    launch_or_warm(warm, k_spmv_sweep_packed<ValueType, T, 2, true, 2, 0, A, false, false, uint32_t *, uint32_t, ValueType *>, grid, block, lds, s, p.d_s_col, \
                   p.d_s_cbase, p.d_s_val, p.d_panel_row, p.d_unit_ent, p.d_unit_panel, p.d_panel_unit, part,        \
                   p.panel_rmax + 1, pcnt, d_x, d_y, (const uint16_t *)nullptr, (const uint8_t *)nullptr,           \
                   (const uint32_t *)nullptr, (const uint32_t *)nullptr, (unsigned long long *)nullptr, 0u,          \
                   (uint32_t)p.nunits, (const A *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, 0u,        \
                   p.y_flag, p.y_epoch, p.y_host)
#define PK(Q, LAG) PKN(true, Q, LAG, 0)
#define PKA(ABL) PKN(true, 2, 2, ABL)
        switch (p.sweep_variant) {
#ifdef SPMV_ABLATIONS
        // measurement variants (tools library): 15/20/22: 2/4/8 groups per barrier; 26-34: loose
        // sync, Q groups, lag (the default is 28: 2 groups, lag 2); 35: the default on the
        // 12-byte rc words of a delta plan
        case 15: PK(2, 0); break;
        case 20: PK(4, 0); break;
        case 22: PK(8, 0); break;
        case 26: PK(4, 1); break;
        case 27: PK(4, 2); break;
        case 29: PK(2, 4); break;
        case 30: PK(2, 1); break;
        case 31: PK(3, 2); break;
        case 32: PK(1, 2); break;
        case 33: PK(1, 4); break;
        case 34: PK(2, 3); break;
        case 35: PK(2, 2); break;
        // measurement-only ablations; 54, 55 and 60-63 give a wrong y by design, DESIGN.md §4
        case 60: if (p.nr_cols >= 32768) { PKA(1); } else { PK(2, 2); } break;  // x gathers all L2 hits
        case 61: PKA(2); break;  // no x gathers
        case 62: PKA(3); break;  // entries from L2 (first 4K of the unit), real gathers
        case 63: if (p.nr_cols >= 32768) { PKA(4); } else { PK(2, 2); } break;  // entries + x from L2
        case 59: PK(2, 1000); break;  // no wave sync (lag never reached)
        case 56: PKN(false, 2, 2, 0); break;  // plain (temporal) entry loads
        case 54: PKA(8); break;  // no LDS adds
        case 55: if (p.nr_cols >= 32768) { PKA(9); } else { PK(2, 2); } break;  // no LDS adds, all L2
        case 57: PKA(6); break;  // x gathers with the nt bit
        case 58: PKA(7); break;  // x gathers that bypass L1 (sc1)
        case 53: PKA(10); break;  // half the value bytes: 8 B/entry streamed instead of 12
        case 50: if (p.panel_rmax >= 16384) { PKA(11); } else { PK(2, 2); } break;  // 11-B entries + delta decode
#endif
        default:
            if (p.sweep_delta) {
#ifdef SPMV_ABLATIONS
                // measurement build: work stealing among a panel's pieces on split plans (the
                // last quarter / half / all of each piece's iterations claimable: variants 39 / 37
                // / 38). Measured 3.5-5.5 % slower than the static split at N = 4 and N = 8
                // (profiles/r04c_steal_ab.jsonl), so the product keeps the static split
                if (p.sweep_steal && (p.sweep_variant == 37 || p.sweep_variant == 38 || p.sweep_variant == 39)) {
                    PKD(true, p.sweep_variant == 37 ? 8 : p.sweep_variant == 38 ? 16 : 4);
                    break;
                }
#endif
                if (p.y_flag || warm) PKDF();  // (warm: load the flagged code object too)
                if (!p.y_flag) PKD(false, 0);
            } else {
                if (p.y_flag || warm) PKF();
                if (!p.y_flag) PK(2, 2);
            }
            break;
        }
#undef PKD
#undef PKDF
#undef PKF
#undef PKA
#undef PK
#undef PKN
        return;
    }
    switch (p.sweep_variant) {
#ifdef SPMV_ABLATIONS
    case 40: SWEEP(4, 1, false, false); break;  // measurement variants of the unpacked form
    case 1: SWEEP(4, 1, false, true); break;
    case 3: SWEEP(4, 1, true, true); break;
    case 7: SWEEP(4, 2, true, true); break;
    case 15: SWEEP(2, 2, true, true); break;
    case 22: SWEEP(2, 8, true, true); break;
#endif
    default: SWEEP(2, 4, true, true); break;  // best unpacked form (0.88 ms on the 10M/160M matrix)
    }
#undef SWEEP
}

// the variants launch_sweep_t sends to the default delta kernel (PKD(false, 0)), split plans
// with the combine kernel: those whose launch can carry the previous step's combine
bool sweep_can_flag_panels(const spmv_plan &p)
{
    if (p.kernel == kKernelBinned)  // pass 2 writes whole panels too (binned.hip k_bin_acc); not
        return p.npanels > 0 && p.variant != 51 && p.variant != 52;  // its ablations
    return p.kernel == kKernelSweep && p.sweep_packed && !p.sweep_det && p.sweep_split == 1 && p.npanels > 0 &&
           (p.sweep_variant == 0 || p.sweep_variant == 28);
}

bool sweep_behind_ok(const spmv_plan &p)
{
    if (!p.sweep_packed || !p.sweep_delta || p.sweep_det || p.sweep_split < 2 || p.d_panel_cnt)
        return false;
    switch (p.sweep_variant) {
    case 15: case 20: case 22: case 26: case 27: case 29: case 30: case 31: case 32: case 33: case 34:
    case 35: case 37: case 38: case 39: case kSweepTurn: case kSweepTurnOrdered:
        return false;
    default:
        return !(p.sweep_variant >= 50 && p.sweep_variant <= 63);
    }
}

template <typename A>
static void launch_sweep_a(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm,
                           int phase, void *part, const sweep_behind &bh)
{
    if (phase != 2) {
        switch (p.sweep_threads) {
        case 256: launch_sweep_t<256, A>(p, d_x, d_y, s, warm, part, bh); break;
        case 512: launch_sweep_t<512, A>(p, d_x, d_y, s, warm, part, bh); break;
        default: launch_sweep_t<1024, A>(p, d_x, d_y, s, warm, part, bh); break;
        }
    }
    if (phase != 1 && p.sweep_split > 1 && !p.d_panel_cnt) {  // the combine kernel (not the fused form)
        const dim3 grid((p.panel_rmax + 255) / 256, (unsigned)p.npanels);
        launch_or_warm(warm, k_sweep_combine<ValueType, A>, grid, dim3(256), 0, s, p.d_panel_row, p.d_panel_unit,
                       reinterpret_cast<const A *>(part), p.panel_rmax + 1, d_y, p.d_steal);
    }
}

hipError_t launch_sweep(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm, int phase,
                        void *part, const sweep_behind *behind)
{
    if (p.npanels == 0)
        return hipSuccess;
    if (!part)
        part = p.d_part;
    const sweep_behind none{};
    if (behind && (behind->cpart || behind->cnext) && !sweep_behind_ok(p))
        return hipErrorNotSupported;
    const sweep_behind &bh = behind ? *behind : none;
    if constexpr (sizeof(ValueType) == 4) {
        if (p.sweep_acc_bytes == 4) {
            launch_sweep_a<float>(p, d_x, d_y, s, warm, phase, part, bh);
            return hipGetLastError();
        }
    }
    launch_sweep_a<double>(p, d_x, d_y, s, warm, phase, part, bh);
    return hipGetLastError();
}

// The pieces of every panel: whole chunks, cut with the even / odd XCC bias d (the weight of
// units [0, u) is u - d (u & 1): the units block-round-robin dispatch sends to even XCCs get
// (1 - d) x the mean, the odd ones (1 + d) x); d = 0 cuts evenly
static void cut_units(const std::vector<uint32_t> &poff, const std::vector<uint32_t> &punit, double d,
                      std::vector<uint32_t> &uent)
{
    const uint32_t P = (uint32_t)punit.size() - 1, U = punit[P];
    uent.assign((size_t)U + 1, 0);
    auto wc = [&](uint32_t u) { return double(u) - d * double(u & 1); };
    for (uint32_t q = 0; q < P; ++q) {
        const uint64_t chunks = (uint64_t(poff[q + 1]) - poff[q]) / kSweepChunk;
        const uint32_t k = punit[q + 1] - punit[q], u0 = punit[q];
        for (uint32_t t = 0; t < k; ++t) {
            const uint64_t c = d != 0.0 ? (uint64_t)(double(chunks) * (wc(u0 + t) - wc(u0)) / (wc(u0 + k) - wc(u0)))
                                        : chunks * t / k;
            uent[u0 + t] = (uint32_t)(poff[q] + kSweepChunk * c);
        }
    }
    uent[U] = poff[P];
}

// Host: panel boundaries (nnz-balanced, <= rmax rows each), then the device sort + scatter.
// Work units: when the slice has at least one panel per resident workgroup, panels are rounded
// to whole rounds of workgroups and each panel is one unit. When it has fewer (a slice of fewer
// than ~5M rows), the panels keep their full LDS size and each is cut into `split` pieces of
// whole chunks of its column-sorted entries (contiguous column ranges, equal entry counts) --
// the reference's 2-D blocking (row slices x column blocks, csr_hw.cpp:25-76) with the column
// blocks sized by work. Denser panels touch fewer x lines per non-zero; the pieces' fp64
// partial sums go to a scratch array and k_sweep_combine adds them per row in piece order
// (env SPMV_SWEEP_SPLIT=0 keeps the smaller-panel form).
int build_sweep(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                hipStream_t s)
{
    const IndexType n = p.nr_rows;
    const uint64_t nnz = p.nnz;
    // a workgroup of T threads gets T/1024 of one CU's LDS for its panel's y
    const uint64_t lds_bytes = kSweepLdsBytes * p.sweep_threads / 1024 - 256;  // 256 B: static LDS
    // accumulator: fp64, or fp32 (compare-and-swap adds) for fp32 matrices with env SPMV_SWEEP_ACC=32
    const char *aenv = ablation_env("SPMV_SWEEP_ACC");
    p.sweep_acc_bytes = sizeof(ValueType) == 4 && aenv && std::atoi(aenv) == 32 ? 4 : 8;
    const uint64_t acc = p.sweep_acc_bytes;
    const uint32_t rmax = (uint32_t)std::min<uint64_t>(lds_bytes / acc - 1, 65534);
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, p.device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
    }
    const int chip_cus = cus;
    cus *= 1024 / p.sweep_threads;  // resident workgroups per round
    // env SPMV_SWEEP_SPLIT: 0 = never split, 2 = split whenever >= 2 pieces fit, else heuristic
    const char *senv = ablation_env("SPMV_SWEEP_SPLIT");
    // env SPMV_SWEEP_DETERMINISTIC=1: the same layout, run by k_spmv_sweep_turn (ordered adds)
    const char *denv = std::getenv("SPMV_SWEEP_DETERMINISTIC");
    const bool det = denv && denv[0] == '1';
    const bool allow_split = !(senv && senv[0] == '0');
    const bool force_split = senv && senv[0] == '2';
    bool split_mode = false;
    // XCC bias: the units the round-robin dispatch sends to even XCCs (unit % 8 even; block b
    // runs on XCC b % 8 in every launch probed, tools/xcc_map_probe.py) get (1 - d) x the mean
    // entries, the odd ones (1 + d) x; weight of the units [0, u): u - d * (u & 1). Why: on the
    // MI355X boxes measured, workgroups on even XCCs sweep 2-4 % slower than on odd ones, in the
    // whole matrix and in the strong-scaling slices (tools/wg_timeline.py,
    // profiles/r03ay_wg_timeline.jsonl, two boxes), and the launch ends with the slowest XCC.
    // Defaults on a whole chip (256 CUs = 8 XCDs): d = 0.015 for whole panels, 0.02 for split
    // pieces (interleaved A/B, profiles/r03bb_xcc_bias.jsonl: 10M/160M -1.3 %, the N = 8 slice
    // -2.0 %, N = 4 -0.7 %); env SPMV_SWEEP_XCC_BIAS=d overrides both (0 = even cut).
    // Split pieces (the N >= 4 strong-scaling slices) are cut evenly by default: which XCCs
    // sweep slower varies from box to box (even ones on the boxes of round 3, odd ones on some of
    // round 4), and the even cut was within 1 % of a per-GPU timed pick and ahead of the fixed
    // 2 % bias at N = 4 (profiles/r04w_xcc_bias_ab.jsonl, r04y), a tie at N = 8. The cut is a
    // function of the matrix and the chip's CU count only, like the reference's (csr_hw.cpp:459-468).
    const char *xbenv = std::getenv("SPMV_SWEEP_XCC_BIAS");
    double xbias_split = xbenv ? std::atof(xbenv) : 0.0;
    double xbias = xbenv ? std::atof(xbenv) : chip_cus == 256 ? 0.015 : 0.0;
    if (!(xbias > -0.5 && xbias < 0.5))
        xbias = xbias_split = 0.0;
    std::vector<uint32_t> prow;
    // subdivide: a run of (nearly) empty rows longer than a panel that no nnz-balanced cut reaches
    // -- most often trailing empty rows -- made every P fail (and the search ran on to P = n);
    // after a bounded search the cuts are taken at the first P and any panel above the LDS rows is
    // split into panels of at most rmax rows
    const uint64_t P_first = std::max<uint64_t>(1, (n + rmax - 1) / rmax);
    uint64_t P_start = P_first;
    // (tools build) SPMV_SWEEP_ROUNDS=k: at least k rounds of whole panels on a matrix that fills
    // a round anyway (smaller panels: earlier first panels for a streamed copy-back)
    if (const char *ke = ablation_env("SPMV_SWEEP_ROUNDS"); ke && std::atoi(ke) > 0 && P_first * 2 >= (uint64_t)cus)
        P_start = std::max<uint64_t>(P_first, (uint64_t)std::min(std::atoi(ke), 8) * cus);
    bool subdivide = false;
    for (uint64_t P = P_start;; ++P) {
        {
            // pieces pay when the slice fills at most half the workgroups with full panels and
            // the partial sums (split * n fp64 values, written once and read once by the
            // combine) stay below 0.6x the entry stream. Measured (profiles/): a 1M-row
            // power-law matrix 14 % faster (partials 0.42x the entries), the N = 8 slice of
            // the 10M/160M matrix 18 % (0.33x), a 300K-row matrix 25 % slower (1.4x)
            const uint64_t S = P ? (uint64_t)cus / P : 0;
            split_mode = !subdivide && allow_split && S >= 2 && P * S * 10 >= (uint64_t)cus * 9 &&
                         (force_split || 2 * S * n * acc * 5 <= 3 * nnz * (4 + sizeof(ValueType)));
        }
        if (!split_mode && P > 1 && P % cus)
            P = (P + cus - 1) / cus * cus;  // whole rounds of workgroups
        P = std::min<uint64_t>(P, std::max<uint64_t>(n, 1));
        prow.assign(1, 0);
        bool ok = true;
        IndexType r = 0;
        for (uint64_t q = 1; q <= P && ok; ++q) {
            const uint64_t target =
                split_mode || xbias == 0.0
                    ? nnz * q / P
                    : (uint64_t)(double(nnz) * (double(q) - xbias * double(q & 1)) / (double(P) - xbias * double(P & 1)));
            IndexType e = (q == P) ? n : (IndexType)(std::lower_bound(h_rp, h_rp + n + 1, (IndexType)target) - h_rp);
            e = std::max(e, r);
            if (e - r > rmax && xbias != 0.0 && !split_mode && q < P)
                e = r + rmax;  // a biased cut past the LDS rows: this panel takes what fits
            if (e - r > rmax && subdivide)
                for (; e - r > rmax; r += rmax)
                    prow.push_back(r + rmax);
            if (e - r > rmax)
                ok = false;
            prow.push_back(e);
            r = e;
        }
        if (ok)
            break;
        if (xbias != 0.0 && !split_mode) {  // the biased cut overflows a panel: cut evenly
            xbias = 0.0;
            --P;
            continue;
        }
        if (P >= n || P > 8 * std::max<uint64_t>(P_first, (uint64_t)cus)) {
            if (subdivide) {
                set_error("build_sweep: cannot form panels");
                return 1;
            }
            subdivide = true;
            xbias = 0.0;
            P = P_start - 1;  // (++P)
        }
    }
    const uint32_t P = (uint32_t)(prow.size() - 1);
    if (split_mode)
        xbias = xbias_split;  // the pieces' cut below (the panels were cut evenly)
    const std::vector<uint32_t> &srow = prow;  // sort segments = the panels
    const uint32_t S = (uint32_t)(srow.size() - 1);
    std::vector<uint32_t> off(S + 1), poff(S + 1);
    off[0] = poff[0] = 0;
    uint32_t rmax_used = 0;
    uint64_t padded = 0;
    for (uint32_t q = 0; q < S; ++q) {
        const uint64_t cnt = uint64_t(h_rp[srow[q + 1]]) - h_rp[srow[q]];
        padded += (cnt + kSweepChunk - 1) / kSweepChunk * kSweepChunk;
        off[q + 1] = (uint32_t)(off[q] + cnt);
        poff[q + 1] = (uint32_t)padded;
    }
    for (uint32_t q = 0; q < P; ++q)
        rmax_used = std::max(rmax_used, prow[q + 1] - prow[q]);
    if (padded > 0xFFFFFFFFull) {  // panel_ent is u32: the padded layout must fit (nnz near 2^32)
        set_error("build_sweep: padded entry count exceeds 32 bits");
        return 2;
    }
    p.npanels = P;
    p.panel_rmax = rmax_used;
    p.ent_pad = poff[S];
    p.sweep_det = det;
    // work units: pieces of whole chunks per panel. split mode: `split` pieces each; any panel
    // with more than twice the mean entry count (a panel holding very long rows) is cut
    // further, so that no workgroup gets more than ~2x the mean work
    uint32_t split = split_mode ? std::max<uint32_t>(1, (uint32_t)cus / P) : 1;
    // env SPMV_SWEEP_PIECES=k (experiments): k pieces per panel in split mode instead of cus / P
    if (const char *kenv = ablation_env("SPMV_SWEEP_PIECES"); split_mode && kenv && std::atoi(kenv) > 0)
        split = (uint32_t)std::atoi(kenv);
    const double mean = P ? double(padded) / P : 0.0;
    std::vector<uint32_t> punit(P + 1, 0);
    for (uint32_t q = 0; q < P; ++q) {
        const uint64_t chunks = (uint64_t(poff[q + 1]) - poff[q]) / kSweepChunk;
        uint64_t k = split * std::max<uint64_t>(
                                 1, (uint64_t)std::ceil(double(poff[q + 1] - poff[q]) / std::max(2.0 * mean, 1.0)));
        k = std::max<uint64_t>(1, std::min<uint64_t>(k, chunks));
        punit[q + 1] = punit[q] + (uint32_t)k;
    }
    const uint32_t U = punit[P];
    std::vector<uint32_t> uent, upanel(std::max<uint32_t>(U, 1));
    bool multi = false;
    for (uint32_t q = 0; q < P; ++q) {
        multi |= punit[q + 1] - punit[q] > 1;
        for (uint32_t u = punit[q]; u < punit[q + 1]; ++u)
            upanel[u] = q;
    }
    cut_units(poff, punit, split_mode ? xbias : 0.0, uent);
    p.xbias_split = split_mode ? xbias : 0.0;
    p.sweep_split = multi ? std::max<uint32_t>(split, 2) : 1;  // > 1: combine kernel needed
    p.nunits = U;
    if (multi) {
        SPMV_TRY(hipMalloc((void **)&p.d_part, (uint64_t)U * (uint64_t(rmax_used) + 1) * acc));
#ifdef SPMV_ABLATIONS
        // work-stealing counters of the measurement variants (zero; every k_sweep_combine re-arms them)
        SPMV_TRY(hipMalloc((void **)&p.d_steal, (uint64_t)U * 8));
        SPMV_TRY(hipMemsetAsync(p.d_steal, 0, (uint64_t)U * 8, s));
#endif
        // env SPMV_SWEEP_COMBINE=fused: the last piece of each panel combines inside the sweep
        // launch instead of k_sweep_combine. Measured slower on the N = 8 slice of the 10M/160M
        // matrix (0.147 vs 0.128 ms, profiles/r03_ab_sweep_combine.jsonl): the panels of a one-round
        // launch all finish together, and each last arriver then reads its 4 x 160 KiB of partials
        // alone (~50-70 GB/s per workgroup, MI355X_MICROARCH.md handoff-payload) where the combine
        // kernel reads them with the whole chip; so the separate launch stays the default
        const char *cenv = ablation_env("SPMV_SWEEP_COMBINE");
        if (cenv && std::strcmp(cenv, "fused") == 0) {
            SPMV_TRY(hipMalloc((void **)&p.d_panel_cnt, std::max<uint64_t>(P, 1) * 4));
            SPMV_TRY(hipMemsetAsync(p.d_panel_cnt, 0, std::max<uint64_t>(P, 1) * 4, s));
        }
    }
    SPMV_TRY(hipMalloc((void **)&p.d_unit_panel, upanel.size() * 4));
    SPMV_TRY(hipMalloc((void **)&p.d_panel_unit, punit.size() * 4));
    SPMV_TRY(hipMemcpyAsync(p.d_unit_panel, upanel.data(), upanel.size() * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMemcpyAsync(p.d_panel_unit, punit.data(), punit.size() * 4, hipMemcpyHostToDevice, s));

    // bucket shift so that S * buckets fits 32-bit keys
    uint32_t shift = 0;
    while ((uint64_t(S) * ((uint64_t(p.nr_cols) >> shift) + 1)) >= (1ull << 32))
        ++shift;
    const uint64_t nbuckets = (uint64_t(p.nr_cols) >> shift) + 1;
    int end_bit = 1;
    while (end_bit < 32 && (1ull << end_bit) < uint64_t(S) * nbuckets)
        ++end_bit;

    SPMV_TRY(hipMalloc((void **)&p.d_panel_row, (P + 1) * 4));
    SPMV_TRY(hipMalloc((void **)&p.d_unit_ent, uent.size() * 4));
    SPMV_TRY(hipMemcpyAsync(p.d_panel_row, prow.data(), (P + 1) * 4, hipMemcpyHostToDevice, s));
    uint32_t *d_srow = p.d_panel_row;  // rows of the sort segments (the panels)
    SPMV_TRY(hipMemcpyAsync(p.d_unit_ent, uent.data(), uent.size() * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMalloc((void **)&p.d_s_col, std::max<uint64_t>(p.ent_pad, 4) * 4));
    SPMV_TRY(hipMalloc((void **)&p.d_s_row, std::max<uint64_t>(p.ent_pad, 4) * 2));
    SPMV_TRY(hipMalloc((void **)&p.d_s_val, std::max<uint64_t>(p.ent_pad, 4) * sizeof(ValueType)));

    uint32_t *d_off = nullptr, *d_poff = nullptr;
    IndexType *d_rp = nullptr;
    uint32_t *k0 = nullptr, *k1 = nullptr, *i0 = nullptr, *i1 = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    uint8_t *d_wide = nullptr;     // per chunk: its columns span >= 65536 (side-table chunk)
    uint32_t *d_abs = nullptr;     // a wide plan's absolute columns, lane-ordered
    auto cleanup = [&]() {
        for (void *q : {(void *)d_off, (void *)d_poff, (void *)d_rp, (void *)k0, (void *)k1, (void *)i0,
                        (void *)i1, tmp, (void *)d_wide, (void *)d_abs})
            if (q)
                (void)hipFree(q);
    };
    auto fail = [&](hipError_t e, const char *what) {
        set_error(std::string("build_sweep: ") + what + ": " + hipGetErrorString(e));
        cleanup();
        return 1;
    };
#define SW_TRY(x)                              \
    do {                                       \
        hipError_t e_ = (x);                   \
        if (e_ != hipSuccess)                  \
            return fail(e_, #x);               \
    } while (0)
    SW_TRY(hipMalloc((void **)&d_off, (S + 1) * 4));
    SW_TRY(hipMalloc((void **)&d_poff, (S + 1) * 4));
    SW_TRY(hipMalloc((void **)&d_rp, (size_t(n) + 1) * 4));
    SW_TRY(hipMemcpyAsync(d_off, off.data(), (S + 1) * 4, hipMemcpyHostToDevice, s));
    SW_TRY(hipMemcpyAsync(d_poff, poff.data(), (S + 1) * 4, hipMemcpyHostToDevice, s));
    SW_TRY(hipMemcpyAsync(d_rp, h_rp, (size_t(n) + 1) * 4, hipMemcpyHostToDevice, s));
    if (nnz) {
        SW_TRY(hipMalloc((void **)&k0, nnz * 4));
        SW_TRY(hipMalloc((void **)&k1, nnz * 4));
        SW_TRY(hipMalloc((void **)&i0, nnz * 4));
        SW_TRY(hipMalloc((void **)&i1, nnz * 4));
        hipLaunchKernelGGL(k_sweep_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_rp, d_col_src,
                           d_srow, S, n, nbuckets, shift, k0, i0);
        SW_TRY(hipGetLastError());
        // 64-bit item count: a slice may hold more than 2^31 non-zeros (up to the 32-bit padded
        // layout checked above)
        SW_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, i0, i1, (uint64_t)nnz, 0, end_bit, s));
        SW_TRY(hipMalloc(&tmp, tmp_bytes));
        SW_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, i0, i1, (uint64_t)nnz, 0, end_bit, s));
        hipLaunchKernelGGL((k_sweep_scatter<ValueType>), dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, k1,
                           i1, nnz, nbuckets, d_rp, n, d_col_src, d_val_src, d_srow, d_off, d_poff,
                           p.d_s_col, p.d_s_row, p.d_s_val);
        SW_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL((k_sweep_pad<ValueType>), dim3((S + 255) / 256), dim3(256), 0, s, S, d_srow, d_off,
                       d_poff, p.d_s_col, p.d_s_row, p.d_s_val);
    SW_TRY(hipGetLastError());
    // 12-byte packed entries when every 128-entry chunk spans < 65536 columns
    {
        const uint32_t group = kSweepChunk, gshift = 7;
        const uint64_t nchunks = p.ent_pad / group;
        SW_TRY(hipMalloc((void **)&p.d_s_cbase, std::max<uint64_t>(nchunks, 1) * 4));
        uint32_t *d_bad = d_off;  // reuse: d_off is no longer needed once the scatter ran
        SW_TRY(hipStreamSynchronize(s));
        SW_TRY(hipMemsetAsync(d_bad, 0, 4, s));
        SW_TRY(hipMalloc((void **)&d_wide, std::max<uint64_t>(nchunks, 1)));
        if (nchunks)
            hipLaunchKernelGGL(k_sweep_chunk_base, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s,
                               p.d_s_col, nchunks, group, p.d_s_cbase, d_bad, d_wide);
        SW_TRY(hipGetLastError());
        uint32_t bad = 0;
        SW_TRY(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, s));
        SW_TRY(hipStreamSynchronize(s));
        const char *env = ablation_env("SPMV_SWEEP_PACKED");
        const bool want = !(env && env[0] == '0');
        const char *lo = ablation_env("SPMV_SWEEP_LANE_ORDER");
        const bool lane = !(lo && lo[0] == '0');
        // the delta-coded entries below (SPMV_SWEEP_DELTA=0 keeps the 12-byte words only).
        // SPMV_SWEEP_DETERMINISTIC=1 plans keep the 12-byte words: the turn kernel on the 11-byte
        // entries measured 0.897 vs 0.871 ms (its deeper pipeline has no room for the decode,
        // profiles/r03_delta_columns.jsonl r03p)
        const char *de = std::getenv("SPMV_SWEEP_DELTA");
        const bool delta = lane && !(de && de[0] == '0') && !det && nchunks && uint64_t(p.nr_cols) < (1ull << 31) &&
                           rmax_used < 32768;
        // a chunk whose columns span >= 65536 has no 16-bit offsets: the delta form carries its
        // absolute columns in the side table (a plan with a few such chunks -- panels of a few
        // entries spread over the columns, e.g. beside a long run of empty rows -- reads only the
        // 11-byte entries). Side chunks stream 15 B per entry, so when more than 1 chunk in 10 is
        // wide (sparse panels throughout), or without the delta form, the plan keeps the
        // unpacked 14-byte entries
        if ((!bad || (delta && uint64_t(bad) * 10 <= nchunks)) && want && p.ent_pad) {
            if (bad) {
                SW_TRY(hipMalloc((void **)&d_abs, p.ent_pad * 4));
                hipLaunchKernelGGL(k_sweep_lane_order_u32, dim3((unsigned)((p.ent_pad + 255) / 256)), dim3(256), 0, s,
                                   p.d_s_col, p.ent_pad, d_abs);
                SW_TRY(hipGetLastError());
                p.sweep_wide = true;
            }
            hipLaunchKernelGGL(k_sweep_pack_rc, dim3((unsigned)((p.ent_pad + 255) / 256)), dim3(256), 0, s, p.d_s_col,
                               p.d_s_row, p.d_s_cbase, p.ent_pad, gshift, d_wide);
            SW_TRY(hipGetLastError());
            SW_TRY(hipStreamSynchronize(s));
            SW_TRY(hipFree(p.d_s_row));
            p.d_s_row = nullptr;
            p.sweep_packed = true;
            if (lane) {
                uint32_t *rc2 = nullptr;
                ValueType *v2 = nullptr;
                SW_TRY(hipMalloc((void **)&rc2, p.ent_pad * 4));
                SW_TRY(hipMalloc((void **)&v2, p.ent_pad * sizeof(ValueType)));
                hipLaunchKernelGGL((k_sweep_lane_order<ValueType>), dim3((unsigned)((p.ent_pad + 255) / 256)), dim3(256),
                                   0, s, p.d_s_col, p.d_s_val, p.ent_pad, rc2, v2);
                SW_TRY(hipGetLastError());
                SW_TRY(hipStreamSynchronize(s));
                SW_TRY(hipFree(p.d_s_col));
                SW_TRY(hipFree(p.d_s_val));
                p.d_s_col = rc2;
                p.d_s_val = v2;
                p.sweep_lane_order = true;
                // delta-coded columns for the default kernel (conditions above)
                if (delta) {
                    uint8_t *d_flag = nullptr;
                    uint32_t *d_sidx = nullptr;
                    SW_TRY(hipMalloc((void **)&p.d_s_row16, p.ent_pad * 2));
                    SW_TRY(hipMalloc((void **)&p.d_s_d8, p.ent_pad));
                    SW_TRY(hipMalloc((void **)&p.d_s_dbase, nchunks * 4));
                    SW_TRY(hipMalloc((void **)&d_flag, nchunks));
                    hipLaunchKernelGGL((k_sweep_delta<ValueType>), dim3((unsigned)((nchunks + 63) / 64)), dim3(64), 0, s,
                                       p.d_s_col, p.d_s_val, nchunks, p.d_s_row16, p.d_s_d8, d_flag, d_wide);
                    hipError_t e = hipGetLastError();
                    std::vector<uint8_t> hf(nchunks);
                    if (e == hipSuccess)
                        e = hipMemcpyAsync(hf.data(), d_flag, nchunks, hipMemcpyDeviceToHost, s);
                    if (e == hipSuccess)
                        e = hipStreamSynchronize(s);
                    (void)hipFree(d_flag);
                    SW_TRY(e);
                    std::vector<uint32_t> sidx(nchunks, 0xFFFFFFFFu);
                    uint64_t ns = 0;
                    for (uint64_t c = 0; c < nchunks; ++c)
                        if (hf[c])
                            sidx[c] = (uint32_t)ns++;
                    p.sweep_side_chunks = ns;
                    SW_TRY(hipMalloc((void **)&p.d_s_side, std::max<uint64_t>(ns, 1) * kSweepChunk * 4));
                    SW_TRY(hipMalloc((void **)&d_sidx, nchunks * 4));
                    e = hipMemcpyAsync(d_sidx, sidx.data(), nchunks * 4, hipMemcpyHostToDevice, s);
                    if (e == hipSuccess) {
                        hipLaunchKernelGGL(k_sweep_delta_base, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s,
                                           p.d_s_col, p.d_s_cbase, d_sidx, nchunks, p.d_s_dbase, p.d_s_side, d_wide,
                                           d_abs);
                        e = hipGetLastError();
                    }
                    if (e == hipSuccess)
                        e = hipStreamSynchronize(s);
                    (void)hipFree(d_sidx);
                    SW_TRY(e);
                    p.sweep_delta = true;
                    // split plans can run the measurement build's work-stealing variants (the separate
                    // combine kernel re-arms the counters)
                    p.sweep_steal = p.sweep_split > 1 && p.d_steal && !p.d_panel_cnt;
                    // the default kernel reads only the 11-byte entries: the rc words are freed
                    // (rebuilt by sweep_materialize_rc for a variant that reads them)
                    SW_TRY(hipFree(p.d_s_col));
                    p.d_s_col = nullptr;
                }
            }
        } else {
            SW_TRY(hipFree(p.d_s_cbase));
            p.d_s_cbase = nullptr;
        }
    }
    SW_TRY(hipStreamSynchronize(s));
#undef SW_TRY
    cleanup();
    return 0;
}

// fraction of sampled rows (with >= 2 entries) whose first two columns lie < 64 apart
int probe_locality(const IndexType *d_rp, const IndexType *d_col, IndexType n, hipStream_t s, double *frac)
{
    *frac = 1.0;
    if (n == 0)
        return 0;
    unsigned long long *d_cnt = nullptr, h[2] = {0, 0};
    SPMV_TRY(hipMalloc((void **)&d_cnt, 16));
    SPMV_TRY(hipMemsetAsync(d_cnt, 0, 16, s));
    const uint32_t stride = std::max<uint32_t>(1, n / 65536);
    const uint64_t threads = (n + stride - 1) / stride;
    hipLaunchKernelGGL(k_locality, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, d_rp, d_col, n, stride,
                       d_cnt);
    SPMV_TRY(hipGetLastError());
    SPMV_TRY(hipMemcpyAsync(h, d_cnt, 16, hipMemcpyDeviceToHost, s));
    SPMV_TRY(hipStreamSynchronize(s));
    SPMV_TRY(hipFree(d_cnt));
    *frac = h[0] ? double(h[1]) / double(h[0]) : 1.0;
    return 0;
}

}  // namespace spmvhw

#ifdef SPMV_ABLATIONS
// measurement build only: copies n words of the workgroup timeline (4 per workgroup) to the host
extern "C" int spmv_abl_wg_times(unsigned long long *out, unsigned n)
{
    if (!out || n > 4 * 4096)
        return 1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(spmvhw::g_abl_wg), size_t(n) * 8, 0, hipMemcpyDeviceToHost) != hipSuccess;
}
#endif

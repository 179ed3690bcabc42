// cg_rast_colour.hip -- rasteriser colour modes 1-2 (randColourSelect,
// rasteriser/Source/skeleton.cpp:647-662): every fragment PixelShader shades
// takes three glibc rand() values, in the reference's fragment order --
// triangle by triangle (:262-281), row by row (:500-508), left to right.
// Which fragments shade depends on the z-buffer at that moment, so the order
// is reconstructed exactly:
//   rast_count_kernel      one wave per row, the ordered z-buffer walk of the
//                          fill: shaded fragments per (triangle, row);
//   rast_scan_rows_kernel  per triangle, exclusive prefix over its rows;
//   rast_scan_tris_kernel  exclusive prefix over triangles (and the total S);
//   rast_rand_kernel       the frame's 3 S rand() values (cg_glibc_rand.h,
//                          jump-ahead to the frame's call offset);
//   rast_fill_rand_kernel  the same walk again, each shaded fragment numbered
//                          (base of its (triangle, row) + rank in the row), the
//                          last one per pixel shaded with its three values.
// The post-pass is shared with colour mode 0 (kStateDirect state).
#include <vector>

#include "cg_glibc_rand.h"
#include "cg_rast_dev.h"

namespace cg {

void *ctx_buf(cg_ctx *c, int which, size_t bytes, hipError_t *e);
int ctx_fail(cg_ctx *c, hipError_t e, const char *what);

constexpr int kRandChunk = 31 * 32;    // rand() values per generator thread

__device__ __forceinline__ RastArgs with_device_light(RastArgs A)
{
    if (A.d_light) {                                      // light from the device geometry (:223)
        const cg_vec4 L = *A.d_light;
        A.light[0] = L.x; A.light[1] = L.y; A.light[2] = L.z;
    }
    return A;
}

// The row's records (lane q holds record base + q) overlapping [x0, x0 + 63].
struct RecLane {
    int lx, rx, shd;
    float lz, sz;
    bool ov;
};
__device__ __forceinline__ RecLane rec_lane(const RowRec *rr, int q, int cnt, int x0)
{
    RecLane r{0, 0, 0, 0.f, 0.f, false};
    if (q < cnt) {
        const RowRec &m = rr[q];
        r.lx = m.lx; r.rx = m.rx; r.lz = m.lz; r.sz = m.sz; r.shd = rec_shadow(m);
        r.ov = !(r.rx - 1 < x0 || r.lx > x0 + 63);
    }
    return r;
}

__global__ __launch_bounds__(64) void rast_count_kernel(RastArgs A, const RowRec *__restrict__ recs,
                                                       const int *__restrict__ count, int *__restrict__ pc)
{
    extern __shared__ int s_cnt[];                        // per record of the row
    const int y = blockIdx.x, lane = threadIdx.x;
    if (y >= A.H) return;
    const int cnt = count[y];
    const RowRec *rr = recs + (size_t)y * A.n;
    for (int i = lane; i < cnt; i += 64) s_cnt[i] = 0;
    __syncthreads();
    for (int x0 = 0; x0 < A.W; x0 += 64) {
        const int x = x0 + lane;
        float depth = 0.0f;                               // :247
        for (int base = 0; base < cnt; base += 64) {
            const RecLane R = rec_lane(rr, base + lane, cnt, x0);
            unsigned long long m = __ballot(R.ov && !R.shd);   // shadow triangles never shade
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1ull;
                const int lx = __builtin_amdgcn_readlane(R.lx, b), rx = __builtin_amdgcn_readlane(R.rx, b);
                const float lz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R.lz), b));
                const float sz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R.sz), b));
                const int i = x - lx;
                const bool in = x < A.W && i >= 0 && x < rx;             // :504, :573
                const float zinv = lz + (sz * (float)i);                 // :543
                const bool pass = in && zinv >= depth;                   // :574
                if (pass) depth = zinv;                                  // :665
                const unsigned long long pm = __ballot(pass);
                if (lane == 0 && pm) s_cnt[base + b] += __popcll(pm);
            }
        }
    }
    __syncthreads();
    for (int i = lane; i < cnt; i += 64) pc[(size_t)rec_t(rr[i]) * A.H + y] = s_cnt[i];
}

// block-wide inclusive scan of v (256 threads); `total` = the block's sum
__device__ __forceinline__ long long block_scan256(long long v, long long &total, long long *s_w)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    long long before = 0;
    total = 0;
    for (int q = 0; q < 4; ++q) {
        const long long x = s_w[q];
        before += q < w ? x : 0;
        total += x;
    }
    __syncthreads();
    return v + before;
}

// per triangle: exclusive prefix of its shaded-fragment counts over its rows
__global__ __launch_bounds__(256) void rast_scan_rows_kernel(const RastHdr *__restrict__ hdr, const int *n_dev,
                                                           int n_cap, int H, int *__restrict__ pc,
                                                           long long *__restrict__ tot)
{
    __shared__ long long s_w[4];
    const int n = n_dev ? min(*n_dev, n_cap) : n_cap;
    for (int t = blockIdx.x; t < n; t += gridDim.x) {
        const RastHdr h = hdr[t];
        long long carry = 0;
        for (int y0 = h.ylo; y0 <= h.yhi; y0 += 256) {
            const int y = y0 + (int)threadIdx.x;
            const long long v = y <= h.yhi ? pc[(size_t)t * H + y] : 0;
            long long chunk;
            const long long inc = block_scan256(v, chunk, s_w);
            if (y <= h.yhi) pc[(size_t)t * H + y] = (int)(carry + inc - v);
            carry += chunk;
        }
        if (threadIdx.x == 0) tot[t] = carry;
    }
}

// exclusive prefix over triangles; total[0] = S, the frame's shaded fragments
__global__ __launch_bounds__(256) void rast_scan_tris_kernel(const long long *__restrict__ tot, const int *n_dev,
                                                           int n_cap, long long *__restrict__ tbase,
                                                           long long *__restrict__ total)
{
    __shared__ long long s_w[4];
    const int n = n_dev ? min(*n_dev, n_cap) : n_cap;
    long long carry = 0;
    for (int t0 = 0; t0 < n; t0 += 256) {
        const int t = t0 + (int)threadIdx.x;
        const long long v = t < n ? tot[t] : 0;
        long long chunk;
        const long long inc = block_scan256(v, chunk, s_w);
        if (t < n) tbase[t] = carry + inc - v;
        carry += chunk;
    }
    if (threadIdx.x == 0) total[0] = carry;
}

// The 61 state words at the frame's first rand() call (cg_glibc_rand.h).
struct RandWindow {
    uint32_t w[61];
};

// Thread b produces values [b C, (b + 1) C) of the frame's stream: its window
// r[idx + b C + j] = sum_i J_b[i] w[i + j] (J_b = x^(b C) mod P), then the
// recurrence r[i] = r[i - 31] + r[i - 3], 31 values per round in registers.
__global__ __launch_bounds__(256) void rast_rand_kernel(RandWindow W, const uint32_t *__restrict__ jt, int nb,
                                                      long long nvals, int32_t *__restrict__ out)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t o[kRandDeg];
#pragma unroll
    for (int j = 0; j < kRandDeg; ++j) o[j] = 0u;
    for (int i = 0; i < kRandDeg; ++i) {
        const uint32_t c = jt[(size_t)b * kRandDeg + i];
#pragma unroll
        for (int j = 0; j < kRandDeg; ++j) o[j] += c * W.w[i + j];
    }
    const long long p0 = (long long)b * kRandChunk;
    for (int m0 = 0; m0 < kRandChunk; m0 += kRandDeg) {
#pragma unroll
        for (int j = 0; j < kRandDeg; ++j)
            if (p0 + m0 + j < nvals) out[p0 + m0 + j] = (int32_t)(o[j] >> 1);      // rand() = r >> 1
        uint32_t nn[kRandDeg];
#pragma unroll
        for (int j = 0; j < kRandDeg; ++j) nn[j] = o[j] + (j < 3 ? o[28 + j] : nn[j - 3]);
#pragma unroll
        for (int j = 0; j < kRandDeg; ++j) o[j] = nn[j];
    }
}

// LO + rand() / (RAND_MAX/HI - LO), all float (skeleton.cpp:563-565, :649-651)
__device__ __forceinline__ float rand_unit(int32_t v)
{
    const float LO = 0.2f, HI = 0.5f;
    const float den = (float)2147483647 / HI - LO;        // RAND_MAX / HI - LO
    return LO + (float)v / den;
}

__global__ __launch_bounds__(64) void rast_fill_rand_kernel(RastArgs A0, const RowRec *__restrict__ recs,
                                                          const int *__restrict__ count, const int *__restrict__ pc,
                                                          const long long *__restrict__ tbase,
                                                          const int32_t *__restrict__ rnd, int mode,
                                                          float4 *__restrict__ state, float *__restrict__ depth_out,
                                                          int32_t *__restrict__ shadow_out)
{
    extern __shared__ long long s_run[];                  // next fragment number per record
    const RastArgs A = with_device_light(A0);
    const int y = blockIdx.x, lane = threadIdx.x;
    if (y >= A.H) return;
    const int cnt = count[y];
    const RowRec *rr = recs + (size_t)y * A.n;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int i = lane; i < cnt; i += 64) {
        const int t = rec_t(rr[i]);
        s_run[i] = tbase[t] + pc[(size_t)t * A.H + y];
    }
    __syncthreads();
    for (int x0 = 0; x0 < A.W; x0 += 64) {
        const int x = x0 + lane;
        float depth = 0.0f;                               // :247
        int shadow = 0, win = -1;                         // :259
        long long widx = 0;
        for (int base = 0; base < cnt; base += 64) {
            const RecLane R = rec_lane(rr, base + lane, cnt, x0);
            unsigned long long m = __ballot(R.ov);
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1ull;
                const int lx = __builtin_amdgcn_readlane(R.lx, b), rx = __builtin_amdgcn_readlane(R.rx, b);
                const float lz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R.lz), b));
                const float sz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(R.sz), b));
                const int shd = __builtin_amdgcn_readlane(R.shd, b);
                const int i = x - lx;
                const bool in = x < A.W && i >= 0 && x < rx;             // :504, :573
                const float zinv = lz + (sz * (float)i);                 // :543
                if (!shd) {
                    const bool pass = in && zinv >= depth;               // :574
                    const unsigned long long pm = __ballot(pass);
                    if (pm) {
                        const long long run = s_run[base + b];
                        if (pass) {
                            depth = zinv;                                // :665
                            win = base + b;
                            widx = run + __popcll(pm & lt);
                        }
                        if (lane == 0) s_run[base + b] = run + __popcll(pm);
                    }
                } else if (in && zinv > depth) {                         // :668-669
                    shadow = 1;
                }
            }
        }
        if (x < A.W) {
            float4 st = make_float4(__int_as_float(-1), 0.f, 0.f, 0.f);
            if (win >= 0) {
                const RowRec r = rr[win];
                const int i = x - r.lx;
                const float X = r.lX + (r.sX * (float)i);                // :547-548 numerators
                const float Y = r.lY + (r.sY * (float)i);
                const cg_vec4 tn = A.tris[rec_t(r)].normal;
                const vec3 D = illum_D(A, depth, X, Y, v3(tn.x, tn.y, tn.z));
                const float r0 = rand_unit(rnd[3 * widx]), r1 = rand_unit(rnd[3 * widx + 1]),
                            r2 = rand_unit(rnd[3 * widx + 2]);
                const vec3 rc = mode == 1 ? v3(r0, r1, r2) : v3(r0 - 0.2f, 1.0f, r2 - 0.2f);   // :652 / :660
                const float ind = A.ind_first;                           // modes 1-2 never rewrite it
                const vec3 sc = rc * (D + v3(ind, ind, ind));
                st = make_float4(__int_as_float(kStateDirect), sc.x, sc.y, sc.z);
            }
            const size_t o = (size_t)y * A.W + x;
            state[o] = st;
            if (depth_out) depth_out[o] = depth;
            shadow_out[o] = shadow;
        }
    }
}

// Host side of colour modes 1-2, between rast_rows_kernel and the post-pass.
// Synchronises once (the stream's length S decides the generator's size).
int rast_colour_fill(cg_ctx *c, const RastArgs &A, const cg_rast_params *p, const RowRec *recs, const int *count,
                     const RastHdr *hdr, const int *n_dev, int max_recs, float4 *state, float *d_depth,
                     int32_t *shadow, hipStream_t st, long long *n_shaded)
{
    hipError_t e;
    const int n = A.n > 0 ? A.n : 1, H = A.H;
    int *pc = (int *)ctx_buf(c, 10, (size_t)n * H * sizeof(int), &e);
    if (!pc) return ctx_fail(c, e, "alloc pass counts");
    long long *tl = (long long *)ctx_buf(c, 11, (2 * (size_t)n + 2) * sizeof(long long), &e);
    if (!tl) return ctx_fail(c, e, "alloc triangle counts");
    long long *tot = tl, *tbase = tl + n, *total = tl + 2 * n;
    if ((e = hipMemsetAsync(pc, 0, (size_t)n * H * sizeof(int), st)) != hipSuccess) return ctx_fail(c, e, "memset");
    const size_t lds_cnt = (size_t)(max_recs > 0 ? max_recs : 1) * sizeof(int);
    hipLaunchKernelGGL(rast_count_kernel, dim3(H), dim3(64), lds_cnt, st, A, recs, count, pc);
    hipLaunchKernelGGL(rast_scan_rows_kernel, dim3(n < 1024 ? n : 1024), dim3(256), 0, st, hdr, n_dev, A.n, H, pc,
                       tot);
    hipLaunchKernelGGL(rast_scan_tris_kernel, dim3(1), dim3(256), 0, st, tot, n_dev, A.n, tbase, total);
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "colour count launch");
    long long S = 0;
    if ((e = hipMemcpyAsync(&S, total, sizeof(S), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ctx_fail(c, e, "shaded-fragment count");
    *n_shaded = S;
    const long long nvals = 3 * S;
    const int nb = (int)((nvals + kRandChunk - 1) / kRandChunk);
    int32_t *rnd = (int32_t *)ctx_buf(c, 12, (size_t)(nvals > 0 ? nvals : 1) * sizeof(int32_t), &e);
    if (!rnd) return ctx_fail(c, e, "alloc rand stream");
    if (nb > 0) {
        // J_b = x^(b C) mod P, grown once per process as frames need more
        static std::vector<uint32_t> jtab;
        static uint32_t step[kRandDeg];
        if (jtab.empty()) {
            rand_poly_xpow(kRandChunk, step);
            jtab.assign(kRandDeg, 0u);
            jtab[0] = 1u;
        }
        while ((int)(jtab.size() / kRandDeg) < nb) {
            uint32_t next[kRandDeg];
            rand_poly_mulmod(&jtab[jtab.size() - kRandDeg], step, next);
            jtab.insert(jtab.end(), next, next + kRandDeg);
        }
        uint32_t *jt = (uint32_t *)ctx_buf(c, 13, (size_t)nb * kRandDeg * sizeof(uint32_t), &e);
        if (!jt) return ctx_fail(c, e, "alloc jump table");
        if ((e = hipMemcpyAsync(jt, jtab.data(), (size_t)nb * kRandDeg * sizeof(uint32_t), hipMemcpyHostToDevice, st)) !=
            hipSuccess)
            return ctx_fail(c, e, "upload jump table");
        RandWindow W;
        rand_window(p->rand_offset, W.w);
        hipLaunchKernelGGL(rast_rand_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, W, jt, nb, nvals, rnd);
    }
    hipLaunchKernelGGL(rast_fill_rand_kernel, dim3(H), dim3(64), (size_t)(max_recs > 0 ? max_recs : 1) * 8, st, A,
                       recs, count, pc, tbase, rnd, p->colour_mode, state, d_depth, shadow);
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "colour fill launch");
    // the jump table upload reads host memory: keep it alive until the copy ran
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return ctx_fail(c, e, "colour fill");
    return CG_OK;
}

}  // namespace cg

// Host-only probe of the restated generator: n values of glibc rand() from
// call `offset` on (seed 1) -- what rast_rand_kernel produces on the device.
extern "C" int cg_glibc_rand(uint64_t offset, int n, int32_t *out)
{
    if (n < 0 || (n && !out)) return CG_E_INVALID;
    uint32_t w[61];
    cg::rand_window(offset, w);
    uint32_t r[cg::kRandDeg];
    for (int j = 0; j < cg::kRandDeg; ++j) r[j] = w[j];
    for (int k = 0; k < n; k += cg::kRandDeg) {
        for (int j = 0; j < cg::kRandDeg && k + j < n; ++j) out[k + j] = (int32_t)(r[j] >> 1);
        uint32_t nn[cg::kRandDeg];
        for (int j = 0; j < cg::kRandDeg; ++j) nn[j] = r[j] + (j < 3 ? r[28 + j] : nn[j - 3]);
        for (int j = 0; j < cg::kRandDeg; ++j) r[j] = nn[j];
    }
    return CG_OK;
}

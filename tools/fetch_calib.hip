// fetch_calib.hip — what rocprofv3's FETCH_SIZE reports for the render kernel's load shapes.
//
// MI355X_MICROARCH.md (HBM section) calibrates FETCH_SIZE only for wide coalesced streaming
// reads (it reports half their bytes) and calls every other access width uncalibrated.  The
// render kernel (rt_mega_kernel) reads:
//   pair   64-B BVH sibling pairs: 4 x global_load_dwordx4 per node lane, one random pair per
//          lane (rt_wavefront.h load_pair / trav_step_coop);
//   tri    48-B triangle records: 3 x dwordx4 per helper lane, a quad of lanes reading 4
//          consecutive records (192 B) of a random leaf (trav_step_coop);
//   texel  4-B texel gathers at random places (rt_path.h tex_sample_ti);
//   stream the guide's calibrated case, coalesced 16 B per lane (control).
// Each kernel below issues one of these shapes over a 2 GiB buffer (8x the 256 MiB Infinity
// Cache), every access in 128-B lines no other access touches (a bijective hash of the access
// index picks the slot), so the bytes asked for and the lines touched are known exactly.  The
// program prints them per kernel as JSON; rocprofv3 --pmc FETCH_SIZE over the same run
// (tools/fetch_calib.sh) gives the counted bytes, and the ratio per shape is the calibration
// bench.py applies (profiles/<tag>_fetch_calib.csv).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

constexpr uint64_t kBytes = 2ull << 30;      // buffer: 2 GiB
constexpr uint64_t kSlot = 256;              // one access (or one quad of tri accesses) per 256-B slot
constexpr uint64_t kSlots = kBytes / kSlot;  // 2^23
constexpr uint32_t kSlotMask = (uint32_t)kSlots - 1u;

// bijection on [0, 2^23): odd multiplier, xor-shift, odd multiplier (mod 2^23)
__device__ __forceinline__ uint32_t perm(uint32_t i) {
    uint32_t x = (i * 0x9E3779B1u) & kSlotMask;
    x ^= x >> 11;
    x = (x * 0x85EBCA77u) & kSlotMask;
    return x;
}

// one 64-B pair per lane: 4 x dwordx4 at a 64-B aligned place in its own slot
__global__ void __launch_bounds__(256) calib_pair(const float4 *__restrict__ buf, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    if (i < n) {
        const float4 *p = buf + (uint64_t)perm(i) * (kSlot / 16) + 4 * (i & 1u);   // offset 0 or 64 in the slot
        const float4 a = p[0], b = p[1], c = p[2], d = p[3];
        s = a.x + b.y + c.z + d.w;
    }
    if (s == 12345.f) out[i] = s;   // (never true on the zeroed buffer: keeps the loads)
}

// quads of lanes: 4 consecutive 48-B records (192 B) of one slot, lane j of the quad reads
// record j with 3 x dwordx4
__global__ void __launch_bounds__(256) calib_tri(const float4 *__restrict__ buf, uint32_t n_quads, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x, q = i >> 2, j = i & 3u;
    float s = 0.f;
    if (q < n_quads) {
        const float4 *p = buf + (uint64_t)perm(q) * (kSlot / 16) + 3 * j;
        const float4 a = p[0], b = p[1], c = p[2];
        s = a.x + b.y + c.z;
    }
    if (s == 12345.f) out[i] = s;
}

// one 4-B word per lane at a random dword of its own slot
__global__ void __launch_bounds__(256) calib_texel(const uint32_t *__restrict__ buf, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    if (i < n) s = (float)buf[(uint64_t)perm(i) * (kSlot / 4) + ((i * 7u) & 31u)];
    if (s == 12345.f) out[i] = s;
}

// coalesced streaming read, 16 B per lane (the guide's calibrated case)
__global__ void __launch_bounds__(256) calib_stream(const float4 *__restrict__ buf, uint64_t n, float *out) {
    float s = 0.f;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const float4 a = buf[i];
        s += a.x + a.w;
    }
    if (s == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = s;
}

// L1/L2 gather rate (not a FETCH_SIZE case: the working set is 2 MiB, L2-resident): every lane
// reads ITER random 64-B pairs as 4 x dwordx4 (the node step's shape: 64 lanes, 64 different
// lines per instruction) ...
constexpr int kIter = 64;
constexpr uint32_t kWin = (2u << 20) / 64;   // pairs in the 2 MiB window
__global__ void __launch_bounds__(256) gather_pair(const float4 *__restrict__ buf, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    uint32_t h = i * 0x9E3779B1u;
    for (int k = 0; k < kIter; ++k) {
        h = h * 1664525u + 1013904223u;
        const float4 *p = buf + 4 * (uint64_t)((h >> 8) & (kWin - 1u));
        const float4 a = p[0], b = p[1], c = p[2], d = p[3];
        s += a.x + b.y + c.z + d.w;
        asm volatile("" : "+v"(s));
    }
    if (s == 12345.f) out[i] = s;
}
// ... the same bytes with the 4 lanes of a quad reading one pair per instruction (lane j its
// float4 j: 16 lines per instruction) ...
__global__ void __launch_bounds__(256) gather_pair_quad(const float4 *__restrict__ buf, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x, j = i & 3u;
    float s = 0.f;
    uint32_t h = (i >> 2) * 0x9E3779B1u;
    for (int k = 0; k < kIter; ++k) {
        h = h * 1664525u + 1013904223u;
        const float4 *p = buf + 4 * (uint64_t)((h >> 8) & (kWin - 1u)) + j;
        const uint32_t h2 = h * 1664525u + 1013904223u, h3 = h2 * 1664525u + 1013904223u,
                       h4 = h3 * 1664525u + 1013904223u;
        const float4 a = p[0], b = buf[4 * (uint64_t)((h2 >> 8) & (kWin - 1u)) + j],
                     c = buf[4 * (uint64_t)((h3 >> 8) & (kWin - 1u)) + j], d = buf[4 * (uint64_t)((h4 >> 8) & (kWin - 1u)) + j];
        h = h4;
        s += a.x + b.y + c.z + d.w;
        asm volatile("" : "+v"(s));
    }
    if (s == 12345.f) out[i] = s;
}
// ... and 4-B random gathers (the texel shape), 4 per iteration
__global__ void __launch_bounds__(256) gather_dword(const uint32_t *__restrict__ buf, float *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    uint32_t h = i * 0x9E3779B1u;
    for (int k = 0; k < kIter; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            h = h * 1664525u + 1013904223u;
            v += buf[(h >> 8) & (kWin * 16u - 1u)];
        }
        s += (float)v;
        asm volatile("" : "+v"(s));
    }
    if (s == 12345.f) out[i] = s;
}

// evicts the caches between shapes: a 512 MiB write
__global__ void __launch_bounds__(256) calib_flush(float4 *buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        buf[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

int main() {
    float4 *buf = nullptr, *junk = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&junk, 512ull << 20));
    CK(hipMalloc(&out, 64u << 20));
    CK(hipMemset(buf, 0, kBytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t n = 1u << 22;   // accesses (pair, texel) or quads (tri): 4 M distinct slots
    std::printf("[\n");
    for (int rep = 0; rep < 2; ++rep) {   // (rep 0 warms the code objects; both are printed)
        struct {
            const char *name;
            double req_bytes, lines;
        } rows[4] = {{"calib_pair", 64.0 * n, 1.0 * n},
                     {"calib_tri", 192.0 * n, 2.0 * n},
                     {"calib_texel", 4.0 * n, 1.0 * n},
                     {"calib_stream", 512.0 * (1 << 20), 512.0 * (1 << 20) / 128.0}};
        for (int k = 0; k < 4; ++k) {
            hipLaunchKernelGGL(calib_flush, dim3(4096), dim3(256), 0, nullptr, junk, (512ull << 20) / 16);
            CK(hipEventRecord(e0, nullptr));
            if (k == 0) hipLaunchKernelGGL(calib_pair, dim3(n / 256), dim3(256), 0, nullptr, buf, n, out);
            if (k == 1) hipLaunchKernelGGL(calib_tri, dim3(4 * n / 256), dim3(256), 0, nullptr, buf, n, out);
            if (k == 2) hipLaunchKernelGGL(calib_texel, dim3(n / 256), dim3(256), 0, nullptr, (const uint32_t *)buf, n, out);
            if (k == 3) hipLaunchKernelGGL(calib_stream, dim3(8192), dim3(256), 0, nullptr, buf, (512ull << 20) / 16, out);
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("  {\"rep\": %d, \"kernel\": \"%s\", \"requested_bytes\": %.0f, \"lines_128b\": %.0f, \"ms\": %.4f, "
                        "\"requested_gbs\": %.1f, \"line_gbs\": %.1f}%s\n",
                        rep, rows[k].name, rows[k].req_bytes, rows[k].lines, ms, rows[k].req_bytes / ms / 1e6,
                        rows[k].lines * 128.0 / ms / 1e6, (rep == 1 && k == 3) ? "" : ",");
        }
    }
    // gather rates: 8 waves per SIMD on every CU (2048 blocks of 256), L2-warm
    int dev = 0, cus = 0, clk_khz = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
    const unsigned gb = (unsigned)cus * 8;
    for (int k = 0; k < 3; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, nullptr));
            if (k == 0) hipLaunchKernelGGL(gather_pair, dim3(gb), dim3(256), 0, nullptr, buf, out);
            if (k == 1) hipLaunchKernelGGL(gather_pair_quad, dim3(gb), dim3(256), 0, nullptr, buf, out);
            if (k == 2) hipLaunchKernelGGL(gather_dword, dim3(gb), dim3(256), 0, nullptr, (const uint32_t *)buf, out);
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double lanes = (double)gb * 256, insts = lanes / 64 * kIter * 4;
            const double lines_per_inst = k == 1 ? 16.0 : 64.0;
            const double cyc = ms * 1e-3 * clk_khz * 1e3;   // at the reported max clock
            std::printf(",\n  {\"rep\": %d, \"kernel\": \"%s\", \"wave_load_insts\": %.0f, \"lines_per_inst\": %.0f, \"ms\": %.4f, "
                        "\"insts_per_cu_cycle\": %.4f, \"line_accesses_per_cu_cycle\": %.4f, \"bytes_per_cu_cycle\": %.2f}",
                        rep, k == 0 ? "gather_pair" : k == 1 ? "gather_pair_quad" : "gather_dword", insts, lines_per_inst, ms,
                        insts / cus / cyc, insts * lines_per_inst / cus / cyc,
                        insts * 64 * (k == 2 ? 4.0 : 16.0) / cus / cyc);
        }
    }
    std::printf("\n]\n");
    CK(hipFree(buf));
    CK(hipFree(junk));
    CK(hipFree(out));
    return 0;
}

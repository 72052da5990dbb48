// rt_device.hip — MI355X (gfx950) render kernels and the device half of the C ABI.
//
// Kernels (SURVEY.md §2 kernel inventory):
//   rt_pixels_kernel      one lane per pixel of the shard, full spp loop in-lane
//                         (replaces Scene::render's OpenMP pixel loop, scene.cpp:31-52)
//   rt_persistent_kernel  persistent lanes pulling pixels from a per-launch atomic
//                         queue (wave-aggregated dequeue), same per-pixel math
// Both write the per-pixel float RGB sum (sample_canvas, scene.cpp:20,42) of the owned
// rows; the result is independent of the kernel, the launch shape and the partition.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <cstdlib>
#include <algorithm>
#include <type_traits>

#include "rt_path.h"
#include "rt_wave.h"
#include "rt_wavefront.h"
#include "rt_mega.h"
#include "rt_quant_lut.h"
#include "rt_scene.h"
#include "rt_bvh_layout.h"

using rtd::Counters;
using rtd::DevScene;

constexpr int kMaxGroups = 8;
struct rt_device_scene {
    int device = -1;
    void *buf = nullptr;         // one allocation holding every array
    DevScene ds{};
    unsigned long long *counters = nullptr;  // 6 x u64
    unsigned int *queue = nullptr;           // persistent kernel work counter
    int cu_count = 0;
    // wavefront path state (allocated on first use, grown on demand)
    void *wf_buf = nullptr;
    long long wf_cap = 0;
    int wf_D = 0;
    rtd::WfState wf{};
    float4 *wf_queue[2] = {nullptr, nullptr};
    float4 *wf_hits = nullptr;
    unsigned *wf_count = nullptr;       // per slot group: [4k] [4k+1] queue counts (active rays)
    unsigned *wf_fetch = nullptr;       // per slot group: kParts extend claim counters
    unsigned *wf_host_count = nullptr;  // pinned, per group
    int wf_groups = 1;                  // slot groups, each on its own stream (RT_WF_GROUPS)
    hipStream_t wf_stream[kMaxGroups] = {};
    hipEvent_t wf_event[kMaxGroups + 1] = {};
    // tuning knobs, environment overrides read at upload (measured values in DESIGN.md §6):
    int wf_refill = 8;                 // RT_WF_REFILL: idle lanes before a wave refills
    int wf_chunk = 64;                 // RT_WF_CHUNK: queue entries claimed per atomic
    int wf_node_lds = 0;               // RT_WF_NODE_LDS: top BVH levels in LDS (measured: no gain)
    double wf_compact_below = 0.75;    // RT_WF_COMPACT_BELOW: dense queue until this active fraction
    int wf_policy = 0;                 // RT_WF_PHASE_POLICY: one of node/leaf steps per iteration (slower)
    int wf_node_cost = 150, wf_leaf_cost = 85;   // RT_WF_NODE_COST / RT_WF_LEAF_COST for that policy
    int wf_xcd = 0;                    // RT_WF_XCD: XCD-affine queue parts in extend (measured slower)
    int wf_ext_bpc = 0;                // RT_WF_EXTEND_BLOCKS_PER_CU: 0 = as many as fit
    int mega_shade_min = 48;           // RT_MEGA_SHADE_MIN: kernel 0 shades once this many lanes are ready
    int mega_trav_min = 0;             // RT_MEGA_TRAV_MIN: ... or once at most this many are traversing
    int mega_wpe = 5;                  // RT_MEGA_WPE: minimum waves per SIMD the register allocation targets
    int mega_reorder = 1;              // RT_MEGA_REORDER: heaviest-first pixel order from the last counting render
    int mega_occ = 0;                  // RT_MEGA_OCC: resident blocks per CU for kernel 0 (0 = occupancy limit)
    int mega_order_min = 3;            // RT_MEGA_ORDER_MIN: reorder only with >= this many pixels per lane
    int mega_tile = 0;                 // RT_MEGA_TILE: heaviest-first by T x T tiles (0 = by pixel)
    int mega_times = 0;                // RT_MEGA_TIMES: diagnostics, per-pixel finish-time percentiles
    int mega_spread = 1;               // RT_MEGA_SPREAD: first pixels of a wave's lanes from different cost strata
    int mega_team = 1;                 // RT_MEGA_TEAM (builds with RT_TEAM=1): a wave's last traversing pixel walked by all its lanes
    int mega_fill = 0;                 // RT_MEGA_FILL: fewer pixels than lanes -> every resident wave, fewer lanes each
    // RT_LIGHT_SPLIT_MIN: light-split kernel (rt_mega.h light_step) from this many emissive
    // triangles (0 = never, the default).  Bit-exact, but measured slower on practice6_1
    // (1,152 lights): -20% at 256x256x4, -13% at 1024x1024x4, -4% at 1920x1080x16
    // (profiles/r01b_light_split_ab.jsonl): the two shading passes per vertex and the walk's
    // extra main-loop iterations cost more than the lockstep walk inside the shading batch.
    int light_split_min = 0;
    unsigned long long *mega_tfin = nullptr;
    long long mega_tfin_n = 0;
    float *fast_part = nullptr;        // fast mode: chunk-major partial sums (chunks x pixels x 3)
    long long fast_part_cap = 0;       // floats
    // that order (per shard geometry): pixel indices by descending traversal work
    int *order = nullptr;
    unsigned *order_cost = nullptr;
    long long order_n = 0, order_cap = 0;
    int order_key[3] = {0, 0, 0};
    bool order_valid = false;
};

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return rt_fail(RT_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ------------------------------------------------------------------------ kernels
using rtd::ShardGeom;
using rtd::shard_row;

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const Counters &c, unsigned long long *out) {
    if (!COUNT) return;
    atomicAdd(&out[0], (unsigned long long)c.rays);
    atomicAdd(&out[1], (unsigned long long)c.aabb);
    atomicAdd(&out[2], (unsigned long long)c.tri);
    atomicAdd(&out[3], (unsigned long long)c.lq);
    atomicAdd(&out[4], (unsigned long long)c.laabb);
    atomicAdd(&out[5], (unsigned long long)c.ltri);
    atomicAdd(&out[6], (unsigned long long)c.hits);
}

template <bool COUNT>
__global__ void __launch_bounds__(256) rt_pixels_kernel(DevScene sc, ShardGeom g, int spp, float *out,
                                                         unsigned long long *counters) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= g.n_pixels) return;
    const int k = (int)(p / g.width), i = (int)(p % g.width);
    const int j = shard_row(g, k);
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    rtv::V3 s = rtd::render_pixel<COUNT>(sc, i, j, spp, cnt);
    out[3 * p + 0] = s.x;
    out[3 * p + 1] = s.y;
    out[3 * p + 2] = s.z;
    flush_counters<COUNT>(cnt, counters);
}

// Persistent variant: grid = resident lanes; each wave takes 64 consecutive pixels per
// dequeue (one returning atomic per wave), so lanes that finish early pick up new work
// without waiting for a block-wide barrier.  Exit: every wave leaves when the queue is
// drained, so the grid always drains.
template <bool COUNT>
__global__ void __launch_bounds__(256) rt_persistent_kernel(DevScene sc, ShardGeom g, int spp, float *out,
                                                             unsigned long long *counters, unsigned int *queue) {
    const int lane = threadIdx.x & 63;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    for (;;) {
        unsigned int base = 0;
        if (lane == 0) base = atomicAdd(queue, 64u);
        base = __shfl(base, 0, 64);
        if ((long long)base >= g.n_pixels) break;
        const long long p = (long long)base + lane;
        if (p < g.n_pixels) {
            const int k = (int)(p / g.width), i = (int)(p % g.width);
            const int j = shard_row(g, k);
            rtv::V3 s = rtd::render_pixel<COUNT>(sc, i, j, spp, cnt);
            out[3 * p + 0] = s.x;
            out[3 * p + 1] = s.y;
            out[3 * p + 2] = s.z;
        }
    }
    flush_counters<COUNT>(cnt, counters);
}

// Wave-synchronous persistent kernel (rt_wave.h): lanes run a flat
// IDLE -> TRAV -> SHADE state machine so a wave never waits for a whole path or pixel.
// Exit: the per-launch queue is monotonic, so once a refill reaches n_pixels the wave
// stops asking; the loop ends when no lane holds a pixel.
template <bool COUNT>
__global__ void __launch_bounds__(256) rt_wave_kernel(DevScene sc, ShardGeom g, int spp, float *out,
                                                       unsigned long long *counters, unsigned int *queue) {
    const int lane = threadIdx.x & 63;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    rtd::Lane L;
    rtd::lane_init(L);
    bool exhausted = false;
    for (;;) {
        // (A) refill: one atomic per wave for all lanes without a pixel
        if (!exhausted) {
            const bool need = L.pix < 0;
            const unsigned long long m = __ballot(need);
            if (m) {
                const int leader = __ffsll((unsigned long long)m) - 1;
                const unsigned cntm = (unsigned)__popcll(m);
                unsigned base = 0;
                if (lane == leader) base = atomicAdd(queue, cntm);
                base = __shfl(base, leader, 64);
                if (need) {
                    const long long p = (long long)base + __popcll(m & ((1ull << lane) - 1ull));
                    if (p < g.n_pixels) rtd::lane_assign(L, sc, g, p);
                }
                if ((long long)base + cntm >= g.n_pixels) exhausted = true;
            }
        }
        if (!__any(L.pix >= 0)) break;
        // (B) IDLE lanes start their next sample
        if (L.pix >= 0 && L.state == rtd::L_IDLE) rtd::lane_start_sample<COUNT>(L, sc, g, cnt);
        // (C) traversal: all traversing lanes step together
        bool trav = L.state == rtd::L_TRAV;
        while (__any(trav)) {
            if (trav) trav = rtd::trav_step<COUNT>(sc, L.r, L.t, L.stk, cnt);
        }
        if (L.state == rtd::L_TRAV) L.state = rtd::L_SHADE;
        // (D) shade, bounce or end the path
        if (L.state == rtd::L_SHADE) rtd::lane_shade<COUNT>(L, sc, spp, out, cnt);
    }
    flush_counters<COUNT>(cnt, counters);
}

// ------------------------------------------------------------------------ frame finish
// Scene::render's last loop (scene.cpp:54-64) on the device: mean, ACES (vector.h:400-407,
// same operation order as rt_tonemap_u8), saturate, then powf(v, 1/2.2) + round(clamp(*255))
// as the exact threshold count of rt_quant_lut.h (glibc powf quantizer, checked monotonic
// over every float in [0, 1] by tools/libm_check.cpp).  NaN gives 0, as on the host.
__constant__ uint32_t k_quant_thr[256];
__global__ void __launch_bounds__(256) rt_finish_kernel(const float *sum, long long n, float normalizer,
                                                         uint8_t *rgb) {
    __shared__ float thr[256];
    thr[threadIdx.x] = __uint_as_float(k_quant_thr[threadIdx.x]);
    __syncthreads();
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        float x = sum[i];
        x *= normalizer;
        const float num = x * (x * 2.51f + 0.03f);
        const float den = x * (x * 2.43f + 0.59f) + 0.14f;
        const float v = rtv::smax(rtv::smin(num / den, 1.f), 0.f);
        int q = 0;
        if (!isnan(v)) {   // #{k in 1..255 : thr[k] <= v}, binary search (thr is non-decreasing)
            int lo = 0;    // invariant: thr[lo] <= v (thr[0] = 0 <= v for v >= 0)
#pragma unroll
            for (int step = 128; step > 0; step >>= 1)
                if (lo + step <= 255 && thr[lo + step] <= v) lo += step;
            q = lo;
        }
        rgb[i] = (uint8_t)q;
    }
}

// ------------------------------------------------------------------------ lane-resident (kernel 4)
// rt_mega.h: every lane runs whole pixels; traversal one unit per iteration, shading batched
// per wave (READY lanes wait for `shade_min` of them or for no lane left traversing).
#ifdef RT_MEGA_PROF
// Diagnostics build (make EXTRA=-DRT_MEGA_PROF): per-wave clock64() split of the main loop.
// [0] shade-iteration cycles [1] traversal-iteration cycles [2] pixel-assign cycles
// [3] shade iterations [4] traversal iterations [5] sum of ready lanes over shade iterations
// [6] sum of traversing lanes over traversal iterations [7] waves
__device__ unsigned long long g_mega_prof[8];
__device__ unsigned long long g_mega_seg[8];   // shading segments (rt_path.h RT_PROF_SEG)
#endif
// FAST (RT_FLAG_FAST): queue items are (chunk, pixel) work units of
// `cs` samples with per-sample Philox seeds; `out` is then the chunk-major partial buffer
// that rt_fast_reduce_kernel folds.
// RT_MEGA_NODE_LDS: traversal reads the top BVH levels from LDS (A/B knob, off)
#ifndef RT_MEGA_NODE_LDS
#define RT_MEGA_NODE_LDS 0
#endif
// LSPLIT: the light pdf's light-BVH walk as a lane state (rt_mega.h light_step), for scenes
// with many emissive triangles (RT_LIGHT_SPLIT_MIN).
template <bool COUNT, int WPE, bool FAST = false, bool LSPLIT = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) rt_mega_kernel(DevScene sc_in, ShardGeom g, rtd::WfState st, int spp, float *out,
                                                       unsigned long long *counters, unsigned int *queue,
                                                       int shade_min, const int *order, unsigned *cost,
                                                       unsigned long long *tfin, int cs = 0) {
    const long long n_items = FAST ? g.n_pixels * (long long)((spp + cs - 1) / cs) : g.n_pixels;
    const int lane = threadIdx.x & 63;
    // texel-decode LUT in LDS: the shading's lane-dependent lookups become ds_reads
    __shared__ float lut[512];
    for (int k = threadIdx.x; k < 512; k += blockDim.x) lut[k] = sc_in.lut[k];
    __syncthreads();
    DevScene sc = sc_in;
    sc.lut = lut;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    uint2 spill[rtd::kStack - rtd::kLdsStack];
#if RT_WIDE
    uint32_t spill_c[rtd::kStack - rtd::kLdsStack];
    rtd::LdsStack3 S{spill, spill_c};
#else
    rtd::LdsStack S{spill};
#endif
#if RT_MEGA_NODE_LDS
    // top kLdsNodes nodes of the breadth-first node array in LDS (rt_wavefront.h LdsNodes)
    const rtd::LdsNodes nodes{sc.node};
    rtd::LdsNodes::fill(sc.node, sc.n_nodes);
#else
    const rtd::GlobalNodes nodes{sc.node};
#endif
    const rtd::NodeRec root = rtd::load_node(rtd::mega_nodes(sc), 0);
    rtd::MegaLane L;
    L.pix = -1;
    L.state = rtd::M_IDLE;
    bool exhausted = false;
    // lanes of the wave that take pixels (bits 16-22 of shade_min; 0 = all 64)
    const int lane_cap = (shade_min >> 16) & 127 ? (shade_min >> 16) & 127 : 64;
    const bool team = (shade_min >> 23) & 1;   // RT_MEGA_TEAM
#ifdef RT_MEGA_PROF
    unsigned long long pf[7] = {0, 0, 0, 0, 0, 0, 0};
    if (threadIdx.x < 8) rt_prof_lds[threadIdx.x] = 0;
    __syncthreads();
    long long tp = clock64();
#endif
    for (;;) {
        if (!exhausted) {   // lanes without a pixel take the next ones (one atomic per wave)
            const bool need = L.pix < 0 && lane < lane_cap;
            const unsigned long long m = __ballot(need);
            if (m) {
                const int leader = __ffsll((unsigned long long)m) - 1;
                const unsigned cm = (unsigned)__popcll(m);
                unsigned base = 0;
                if (lane == leader) base = atomicAdd(queue, cm);
                base = __shfl(base, leader, 64);
                if (need) {
                    const long long p = (long long)base + __popcll(m & ((1ull << lane) - 1ull));
                    if (p < n_items) {
                        if (FAST) rtd::mega_assign_fast<COUNT>(L, sc, g, p, cs, spp, root, cnt);
                        else rtd::mega_assign<COUNT>(L, sc, g, order ? order[p] : (int)p, root, cnt);
                    }
                }
                if ((long long)base + cm >= n_items) exhausted = true;

            }
        }
        if (!__any(L.pix >= 0)) break;
        const int nr = __popcll(__ballot(L.state == rtd::M_READY || (LSPLIT && L.state == rtd::M_LREADY)));
        const int nt = __popcll(__ballot(L.state == rtd::M_TRAV || (LSPLIT && L.state == rtd::M_LTRAV)));
        // shade_min: low byte = ready lanes that trigger a shading pass; next byte = shade
        // anyway once no more than this many lanes are still traversing
        const bool shade_now = nr > 0 && (nr >= (shade_min & 255) || nt <= ((shade_min >> 8) & 255));
#if RT_TEAM && !RT_WIDE
        // the wave's last pixel is traversing: the whole wave walks its ray (rt_team.h)
        if (!COUNT && team && nt == 1 && nr == 0) {
            const unsigned long long act = __ballot(L.pix >= 0);
#ifdef RT_MEGA_PROF
            const long long t0 = clock64();
#endif
            if (__popcll(act) == 1 && rtd::mega_team(L, __ffsll((unsigned long long)act) - 1, sc)) {
#ifdef RT_MEGA_PROF
                tp = clock64();
                if (lane == 0) {
                    atomicAdd(&rt_prof_lds[6], (unsigned long long)(tp - t0));
                    atomicAdd(&rt_prof_lds[7], 1ull);
                }
#endif
                continue;
            }
        }
#endif
#ifdef RT_MEGA_PROF
        {
            const long long t1 = clock64();
            pf[2] += (unsigned long long)(t1 - tp);
            tp = t1;
            pf[shade_now ? 3 : 4] += 1;
            pf[shade_now ? 5 : 6] += (unsigned long long)(shade_now ? nr : nt);
        }
#endif
        if (FAST || LSPLIT) {
            rtd::mega_iterate<COUNT, decltype(S), decltype(nodes), FAST, LSPLIT>(L, shade_now, sc, g, st, spp, out, cost,
                                                                               root, S, nodes, cnt);
        } else if (COUNT && tfin) {   // diagnostics (RT_MEGA_TIMES, counting renders only)
            const long long pix_before = L.pix;
            rtd::mega_iterate<COUNT>(L, shade_now, sc, g, st, spp, out, cost, root, S, nodes, cnt);
            if (pix_before >= 0 && L.pix < 0) tfin[pix_before] = wall_clock64();
        } else {
            rtd::mega_iterate<COUNT>(L, shade_now, sc, g, st, spp, out, cost, root, S, nodes, cnt);
        }
#ifdef RT_MEGA_PROF
        {
            const long long t1 = clock64();
            pf[shade_now ? 0 : 1] += (unsigned long long)(t1 - tp);
            tp = t1;
        }
#endif
    }
#ifdef RT_MEGA_PROF
    if (lane == 0) {
        for (int k = 0; k < 7; ++k) atomicAdd(&g_mega_prof[k], pf[k]);
        atomicAdd(&g_mega_prof[7], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < 8) atomicAdd(&g_mega_seg[threadIdx.x], rt_prof_lds[threadIdx.x]);
#endif
    flush_counters<COUNT>(cnt, counters);
}

// Fast mode: pixel sum = partials of chunks 0, 1, ... added in order (deterministic; the
// oracle's rt_oracle_render_fast adds them the same way).  part is chunk-major: n3 floats
// per chunk.
__global__ void __launch_bounds__(256) rt_fast_reduce_kernel(const float *__restrict__ part, float *__restrict__ out,
                                                             long long n3, int chunks) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n3) return;
    float s = 0.f;
    for (int c = 0; c < chunks; ++c) s += part[(long long)c * n3 + i];
    out[i] = s;
}

// ------------------------------------------------------------------------ wavefront
// (rt_wavefront.h) init -> { extend ; shade } until every slot has finished its samples.
// Queue modes.  Dense: entry p holds slot (slot0 + p)'s ray, or an inactive marker (slot
// -1) once that pixel has all its samples; the order never changes, so a wave's lanes keep
// neighbouring pixels (coherent camera rays, coalesced slot-state access) for the whole
// frame.  Compact: active rays only, appended with one atomic per wave; used for the tail
// of the frame, when most slots are finished.  In both modes *count is the number of
// active rays (the host's termination test).
__global__ void __launch_bounds__(256) wf_init_kernel(DevScene sc, ShardGeom g, rtd::WfState st, long long i0,
                                                       long long i1, float4 *qout, unsigned *cout) {
    for (long long base = i0 + (long long)blockIdx.x * blockDim.x; base < i1; base += (long long)gridDim.x * blockDim.x) {
        const long long i = base + threadIdx.x;
        const bool valid = i < i1;
        if (valid) rtd::store_qray(sc, qout, (unsigned)(i - i0), (int)i, rtd::wf_init_slot(sc, g, st, i));
        rtd::queue_slot(valid, cout);   // active count
    }
}

// Persistent traversal over the queue: each loop iteration advances every lane of a wave
// by one unit of its own ray's traversal (rt_wavefront.h trav_step: one node pair or one
// triangle).  Lanes whose ray is finished idle until `refill` of them are idle (or the
// wave has nothing else to do), then take the next rays of the wave's current chunk of the
// queue; a wave claims a new chunk of `chunk` entries with one atomic when its chunk runs
// out (a single shared counter hit by every refill serialises all waves on one address).
// The rays sit in the queue entries: one coalesced load each.
constexpr unsigned kParts = 8;   // extend queue parts (XCDs)
template <bool COUNT, bool NODE_LDS>
__global__ void __launch_bounds__(256) wf_extend_kernel(DevScene sc, const float4 *qin, const unsigned *count,
                                                         unsigned npos, float4 *hits, unsigned *fetch,
                                                         unsigned *next_count, unsigned long long *counters, int refill,
                                                         unsigned chunk, int policy, int policy_node_cost,
                                                         int policy_leaf_cost, int xcd_parts) {
    const unsigned n = npos ? npos : *count;   // queue positions (dense: all slots of the group)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&counters[7], (unsigned long long)n);  // rays extended
        *next_count = 0;                                 // the shade kernel's output queue
    }
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    uint2 spill[rtd::kStack - rtd::kLdsStack];
    rtd::LdsStack S{spill};
    const int lane = threadIdx.x & 63;
    using Nodes = typename std::conditional<NODE_LDS, rtd::LdsNodes, rtd::GlobalNodes>::type;
    if (NODE_LDS) rtd::LdsNodes::fill(sc.node, sc.n_nodes);
    const Nodes nodes{sc.node};
    const rtd::NodeRec root = rtd::load_node(sc.node, 0);
    unsigned q = 0, lo = 0, hi = 0;   // [lo, hi): the wave's unclaimed part of its chunk
    // XCD affinity: the queue is cut into kParts contiguous parts (dense queue = pixel bands);
    // blocks sharing an XCD (blockIdx % 8, MI355X_MICROARCH.md) drain their own part first,
    // so an XCD's L2 holds the BVH region of its band's rays, then help the other parts.
    const unsigned home = xcd_parts ? blockIdx.x % kParts : 0;
    unsigned part_i = 0;   // parts tried so far, in order home, home+1, ...
    const unsigned nparts = xcd_parts ? kParts : 1;
    bool busy = false, exhausted = false;
    rtd::Ray r;
    rtd::TravState T;
    for (;;) {
        const unsigned long long m = __ballot(!busy);
        const unsigned idle = (unsigned)__popcll(m);
        if (!exhausted && (idle >= (unsigned)refill || idle == 64)) {
            const unsigned rank = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            unsigned got = 0, mine = 0xffffffffu;
            while (got < idle) {
                if (lo >= hi) {
                    while (part_i < nparts) {
                        const unsigned part = (home + part_i) % nparts;
                        const unsigned p0 = (unsigned)((unsigned long long)n * part / nparts);
                        const unsigned p1 = (unsigned)((unsigned long long)n * (part + 1) / nparts);
                        unsigned b = 0;
                        if (lane == 0) b = atomicAdd(&fetch[part], chunk);
                        b = __shfl(b, 0, 64);
                        if (p0 + b < p1) {
                            lo = p0 + b;
                            hi = lo + chunk < p1 ? lo + chunk : p1;
                            break;
                        }
                        ++part_i;
                    }
                    if (part_i >= nparts) {
                        exhausted = true;
                        break;
                    }
                }
                const unsigned k = hi - lo < idle - got ? hi - lo : idle - got;
                if (!busy && rank >= got && rank < got + k) mine = lo + (rank - got);
                lo += k;
                got += k;
            }
            if (mine != 0xffffffffu) {
                q = mine;
                uint32_t bits;
                int slot;
                r = rtd::load_qray_trav(qin, q, bits, slot);
                if (slot >= 0) {   // (dense queue: inactive entries are skipped)
                    busy = rtd::trav_start<COUNT>(bits, root.a, root.b, T, cnt);
                    if (!busy) rtd::store_hit(hits, q, T.best);   // misses the scene box
                }
            }
        }
        // phase choice: lanes at internal nodes and lanes at leaf triangles run different
        // code; with policy != 0 a wave runs only one of the two per iteration (the one with
        // more useful lanes per instruction) and the other lanes wait, instead of paying for
        // both branches every iteration.
        bool step = busy;
        if (policy) {
            const int nn = __popcll(__ballot(busy && T.phase == rtd::TP_NODE));
            const int nl = __popcll(__ballot(busy && T.phase == rtd::TP_LEAF));
            const bool do_node = nn * policy_leaf_cost >= nl * policy_node_cost;
            step = busy && ((T.phase == rtd::TP_NODE) == do_node);
        }
        if (step && rtd::trav_step<COUNT>(sc, r, T, S, nodes, cnt)) {
            rtd::store_hit(hits, q, T.best);
            busy = false;
        }
        if (exhausted && !__any(busy)) break;
    }
    rtd::counters_flush<COUNT>(cnt, counters);
}

// Per-block LDS copies of the small tables every shading hit reads with a lane-dependent
// index (texel decode LUT, materials): LDS reads instead of divergent vector-memory gathers.
constexpr int kMatLds = 64;
struct ShadeLds {
    float lut[512];
    float mf[kMatLds * 12];
    int mt[kMatLds * 4];
    double nt[kMatLds * 16];
};

template <bool COUNT, bool MAT_LDS>
__global__ void __launch_bounds__(256) wf_shade_kernel(DevScene sc_in, ShardGeom g, rtd::WfState st, int spp,
                                                        const float4 *qin, const unsigned *cin, unsigned npos,
                                                        const float4 *hits, float4 *qout, unsigned *cout,
                                                        long long slot0, int dense_out, unsigned *fetch, float *out,
                                                        unsigned long long *counters) {
    __shared__ ShadeLds L;
    for (int k = threadIdx.x; k < 512; k += blockDim.x) L.lut[k] = sc_in.lut[k];
    if (MAT_LDS) {
        for (int k = threadIdx.x; k < sc_in.n_meshes * 12; k += blockDim.x) L.mf[k] = sc_in.mesh_f[k];
        for (int k = threadIdx.x; k < sc_in.n_meshes * 4; k += blockDim.x) L.mt[k] = sc_in.mesh_tex[k];
        for (int k = threadIdx.x; k < sc_in.n_meshes * 16; k += blockDim.x) L.nt[k] = sc_in.mesh_nt[k];
    }
    __syncthreads();
    DevScene sc = sc_in;
    sc.lut = L.lut;
    if (MAT_LDS) {
        sc.mesh_f = L.mf;
        sc.mesh_tex = L.mt;
        sc.mesh_nt = L.nt;
    }
    const unsigned n = npos ? npos : *cin;   // input positions (dense: all slots of the group)
    if (blockIdx.x == 0 && threadIdx.x < kParts) fetch[threadIdx.x] = 0;   // the next extend launch's ray counters
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    for (unsigned base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const unsigned q = base + threadIdx.x;
        int slot = -1;
        bool next = false;
        rtd::Ray r;
        if (q < n) {
            r = rtd::load_qray(qin, q, slot);
            if (slot >= 0) {
                const rtd::Hit h = rtd::load_hit(hits, q);
                next = rtd::wf_shade_slot<COUNT>(sc, g, st, spp, slot, r, h, out, cnt);
            }
        }
        const unsigned p = rtd::queue_slot(next, cout);
        if (dense_out) {   // (dense out implies dense in: entry q is slot slot0 + q)
            if (next) rtd::store_qray(sc, qout, q, slot, r);
            else if (q < n) rtd::store_qray_inactive(qout, q);
        } else if (next) {
            rtd::store_qray(sc, qout, p, slot, r);
        }
    }
    rtd::counters_flush<COUNT>(cnt, counters);
}

// Ray-level entry: BVH::intersect + ManyLightsDistribution::pdf for explicit rays.
__global__ void __launch_bounds__(256) rt_rays_kernel(DevScene sc, long long n, const float *org, const float *dir,
                                                       float *out_f, long long *out_i) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    rtd::Ray r = rtd::make_ray(rtv::V3{org[3 * k], org[3 * k + 1], org[3 * k + 2]},
                               rtv::V3{dir[3 * k], dir[3 * k + 1], dir[3 * k + 2]});
    Counters c1{0, 0, 0, 0, 0, 0, 0}, c2{0, 0, 0, 0, 0, 0, 0};
    rtd::Hit h;
    const bool ok = rtd::closest_hit<true>(sc, r, h, c1);
    const float lp = sc.n_lights ? rtd::light_pdf<true>(sc, r.o, r.d, c2) : 0.f;
    out_f[4 * k + 0] = ok ? h.t : 0.f;
    out_f[4 * k + 1] = ok ? h.u : 0.f;
    out_f[4 * k + 2] = ok ? h.v : 0.f;
    out_f[4 * k + 3] = lp;
    out_i[6 * k + 0] = ok;
    out_i[6 * k + 1] = ok ? h.prim : -1;
    out_i[6 * k + 2] = c1.aabb;
    out_i[6 * k + 3] = c1.tri;
    out_i[6 * k + 4] = c2.laabb;
    out_i[6 * k + 5] = c2.ltri;
}

// ------------------------------------------------------------------------ host side
namespace {

template <class T>
size_t append(std::vector<uint8_t> &blob, const std::vector<T> &v, size_t pre = 0) {
    size_t off = ((blob.size() + 255) & ~size_t(255)) + pre;
    blob.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

// The device copies of the scene BVH are renumbered breadth-first (rt_bvh_layout.h): a
// node's children stay an adjacent pair (right = left + 1) and leaves keep their triangle
// ranges, so traversal visits, counters and results are unchanged; the wide copy adds the
// near-child prefetch word of rt_trav_wide.h.
using rtd::bfs_nodes;

// Device texture layout: texture t's texels in 4x4 tiles, tile (tx, ty) at tile index
// ty * ceil(w/4) + tx, texel (x & 3, y & 3) at 4 * (y & 3) + (x & 3) inside it; tex_info keeps
// (offset in texels, width, height, channels).
void tile_textures(const std::vector<uint32_t> &info, const std::vector<uint8_t> &texels, std::vector<uint32_t> &info_out,
                   std::vector<uint32_t> &out) {
    const size_t n = info.size() / 4;
    info_out = info;
    out.clear();
    for (size_t t = 0; t < n; ++t) {
        const uint32_t off = info[4 * t], w = info[4 * t + 1], h = info[4 * t + 2];
        const uint32_t tw = (w + 3) / 4, th = (h + 3) / 4;
        const size_t base = out.size();
        info_out[4 * t] = (uint32_t)base;
        out.resize(base + (size_t)tw * th * 16, 0u);
        for (uint32_t y = 0; y < h; ++y)
            for (uint32_t x = 0; x < w; ++x) {
                uint32_t v;
                std::memcpy(&v, &texels[4 * ((size_t)off + (size_t)y * w + x)], 4);
                out[base + ((size_t)(y >> 2) * tw + (x >> 2)) * 16 + (y & 3) * 4 + (x & 3)] = v;
            }
    }
}

int ensure_device_scene(rt_scene *s, int device) {
    if (s->dev && s->dev->device == device) return RT_OK;
    if (s->dev) rt_device_scene_release(s);
    if (s->bvh_depth + 2 >= (uint32_t)rtd::kStack || s->light_bvh_depth + 2 >= (uint32_t)rtd::kStack)
        return rt_fail(RT_ERR_LIMIT, "BVH deeper than the device traversal stack (" + std::to_string(rtd::kStack) + ")");
    if (s->ray_depth > rtd::kMaxDepth) return rt_fail(RT_ERR_LIMIT, "ray_depth exceeds device limit");
    for (size_t k = 0; k < s->node.size() / 8; ++k) {  // wavefront traversal frame packing (rt_wavefront.h)
        uint32_t a, b;
        std::memcpy(&a, &s->node[8 * k + 6], 4);
        std::memcpy(&b, &s->node[8 * k + 7], 4);
        if (a >= rtd::kFrameMaxA || b >= 1024u)
            return rt_fail(RT_ERR_LIMIT, "scene too large for the device BVH frame packing (2^22 nodes/triangles, 255 per leaf)");
    }
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return rt_fail(RT_ERR_DEVICE, "no HIP device " + std::to_string(device));
    HIP_TRY(hipSetDevice(device));
    std::vector<uint8_t> blob;
    const std::vector<float> bfs = bfs_nodes(s->node);
    std::vector<float> wide;
    try {
        wide = rtd::wide_nodes(bfs);
    } catch (const std::exception &ex) {
        return rt_fail(RT_ERR_LIMIT, ex.what());
    }
    // (every array starts 256-B aligned: a leaf lane's 4 x 16-B read of the last triangle
    // stays inside the allocation)
    const size_t o_tri = append(blob, s->tri), o_attr = append(blob, s->tri_attr), o_tan = append(blob, s->tri_tan),
                 o_node = append(blob, bfs, 32), o_light = append(blob, s->light),
                 o_node_w = append(blob, wide, 32),
                 o_lnode = append(blob, s->light_node), o_mf = append(blob, s->mesh_f),
                 o_mt = append(blob, s->mesh_tex), o_nt = append(blob, s->mesh_nt);
    // textures in 4x4-texel tiles (64 B, one cache line): a bilinear 2x2 footprint usually
    // stays in one line instead of always spanning two rows (rt_path.h tex_sample)
    std::vector<uint32_t> tinfo, tiled;
    tile_textures(s->tex_info, s->texels, tinfo, tiled);
    const size_t o_ti = append(blob, tinfo), o_tx = append(blob, tiled);
    std::vector<float> lut(512);
    rtd::fill_decode_lut(lut.data());
    const size_t o_lut = append(blob, lut);
    // node array at +32 B: sibling pairs (left odd, left + 1) share one 64-B line
    blob.resize(((blob.size() + 255) & ~size_t(255)) + 256);
    rt_device_scene *d = new rt_device_scene();
    d->device = device;
    hipError_t e = hipMalloc(&d->buf, blob.size());
    if (e == hipSuccess) e = hipMemcpy(d->buf, blob.data(), blob.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&d->counters, 8 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void **)&d->queue, 64);
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        if (d->buf) (void)hipFree(d->buf);
        if (d->counters) (void)hipFree(d->counters);
        if (d->queue) (void)hipFree(d->queue);
        delete d;
        return rt_fail(RT_ERR_DEVICE, std::string("scene upload: ") + hipGetErrorString(e));
    }
    d->cu_count = prop.multiProcessorCount;
    if (const char *e = std::getenv("RT_WF_REFILL")) d->wf_refill = std::max(1, std::min(64, std::atoi(e)));
    if (const char *e = std::getenv("RT_WF_CHUNK")) d->wf_chunk = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("RT_WF_NODE_LDS")) d->wf_node_lds = std::atoi(e) != 0;
    if (const char *e = std::getenv("RT_WF_COMPACT_BELOW")) d->wf_compact_below = std::atof(e);
    if (const char *e = std::getenv("RT_WF_PHASE_POLICY")) d->wf_policy = std::atoi(e);
    if (const char *e = std::getenv("RT_WF_XCD")) d->wf_xcd = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_SHADE_MIN")) d->mega_shade_min = std::min(64, std::max(1, std::atoi(e)));
    if (const char *e = std::getenv("RT_MEGA_TRAV_MIN")) d->mega_trav_min = std::min(64, std::max(0, std::atoi(e)));
    if (const char *e = std::getenv("RT_MEGA_WPE")) d->mega_wpe = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_REORDER")) d->mega_reorder = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_OCC")) d->mega_occ = std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_MEGA_ORDER_MIN")) d->mega_order_min = std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_MEGA_TILE")) d->mega_tile = std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_MEGA_TIMES")) d->mega_times = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_SPREAD")) d->mega_spread = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_FILL")) d->mega_fill = std::atoi(e);
    if (const char *e = std::getenv("RT_MEGA_TEAM")) d->mega_team = std::atoi(e);
    if (const char *e = std::getenv("RT_LIGHT_SPLIT_MIN")) d->light_split_min = std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_WF_NODE_COST")) d->wf_node_cost = std::atoi(e);
    if (const char *e = std::getenv("RT_WF_LEAF_COST")) d->wf_leaf_cost = std::atoi(e);
    if (const char *e = std::getenv("RT_WF_GROUPS")) d->wf_groups = std::max(1, std::min(kMaxGroups, std::atoi(e)));
    if (const char *e = std::getenv("RT_WF_EXTEND_BLOCKS_PER_CU")) d->wf_ext_bpc = std::max(0, std::atoi(e));
    uint8_t *b = (uint8_t *)d->buf;
    DevScene &ds = d->ds;
    ds.tri = (const float4 *)(b + o_tri);
    ds.tri_attr = (const float4 *)(b + o_attr);
    ds.tri_tan = (const float4 *)(b + o_tan);
    ds.node = (const float4 *)(b + o_node);
    ds.node_w = (const float4 *)(b + o_node_w);
    ds.light = (const float4 *)(b + o_light);
    ds.light_node = (const float4 *)(b + o_lnode);
    ds.mesh_f = (const float *)(b + o_mf);
    ds.mesh_tex = (const int *)(b + o_mt);
    ds.mesh_nt = (const double *)(b + o_nt);
    ds.tex_info = (const uint4 *)(b + o_ti);
    ds.texels = (const uint32_t *)(b + o_tx);
    ds.lut = (const float *)(b + o_lut);
    ds.n_lights = (int)(s->light.size() / 16);
    ds.n_tris = (int)(s->tri.size() / 12);
    ds.n_nodes = (int)(s->node.size() / 8);
    ds.n_meshes = (int)(s->mesh_f.size() / 12);
    ds.ray_depth = s->ray_depth;
    ds.max_distance = s->max_distance;
    ds.width = s->width;
    ds.height = s->height;
    std::memcpy(ds.cam_pos, s->cam_pos, sizeof ds.cam_pos);
    std::memcpy(ds.cam_axes, s->cam_axes, sizeof ds.cam_axes);
    std::memcpy(ds.tan_fov, s->tan_half_fov, sizeof ds.tan_fov);
    s->dev = d;
    return RT_OK;
}

// Wavefront workspace: SoA path state for `n` slots with `D` vertex records each.
int ensure_wf(rt_device_scene *d, long long n, int D) {
    if (d->wf_buf && d->wf_cap >= n && d->wf_D == D) return RT_OK;
    if (d->wf_buf) (void)hipFree(d->wf_buf);
    if (d->wf_count) (void)hipFree(d->wf_count);
    if (d->wf_host_count) (void)hipHostFree(d->wf_host_count);
    d->wf_buf = nullptr;
    d->wf_count = nullptr;
    d->wf_host_count = nullptr;
    const long long cap = ((n + 255) / 256) * 256;
    const int planes = 8 + 9 * D + 20         // slot state (2 x 16 B), vertex records (36 B each), light-split mid (80 B)
                       + 2 * 4 * rtd::kQRec + 4;   // two ray queues (48 B / entry), hits (16 B / entry)
    const size_t bytes = (size_t)cap * 4 * (size_t)planes;
    HIP_TRY(hipMalloc(&d->wf_buf, bytes));
    HIP_TRY(hipMalloc((void **)&d->wf_count, 16 * kMaxGroups));
    if (!d->wf_fetch) HIP_TRY(hipMalloc((void **)&d->wf_fetch, sizeof(unsigned) * kParts * kMaxGroups));
    HIP_TRY(hipHostMalloc((void **)&d->wf_host_count, 16 * kMaxGroups, hipHostMallocDefault));
    for (int k = 0; k < d->wf_groups; ++k)
        if (!d->wf_stream[k]) HIP_TRY(hipStreamCreateWithFlags(&d->wf_stream[k], hipStreamNonBlocking));
    for (int k = 0; k <= d->wf_groups; ++k)
        if (!d->wf_event[k]) HIP_TRY(hipEventCreateWithFlags(&d->wf_event[k], hipEventDisableTiming));
    float *f = (float *)d->wf_buf;
    auto take = [&](long long k) { float *p = f; f += (size_t)cap * k; return p; };
    rtd::WfState &w = d->wf;
    w.n = n;
    w.D = D;
    d->wf_queue[0] = (float4 *)take(4 * rtd::kQRec);   // 16-B aligned: cap is a multiple of 256
    d->wf_queue[1] = (float4 *)take(4 * rtd::kQRec);
    d->wf_hits = (float4 *)take(4);
    w.st = (float4 *)take(8);
    w.rec_ab = (float4 *)take(8 * D);
    w.rec_c = take(D);
    w.mid = (float4 *)take(20);   // 5 planes of float4, stride = lane slots (<= cap)
    d->wf_cap = cap;
    d->wf_D = D;
    return RT_OK;
}

template <class K>
unsigned persistent_blocks(rt_device_scene *d, K kernel, long long work, int cap_per_cu = 0) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    if (cap_per_cu > 0 && per_cu > cap_per_cu) per_cu = cap_per_cu;
    long long need = (work + 255) / 256;
    long long b = std::min<long long>(need, (long long)d->cu_count * per_cu);
    return (unsigned)std::max<long long>(b, 1);
}

// Per-launch HIP events for RT_FLAG_KERNEL_TIMES.
struct LaunchTimer {
    bool on = false;
    std::vector<hipEvent_t> ev[2];   // [kernel]: start, end, start, end, ...
    hipError_t mark(int k, hipStream_t s) {
        if (!on) return hipSuccess;
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        ev[k].push_back(e);
        return hipEventRecord(e, s);
    }
    // sums the durations (after the stream has drained) and releases the events
    hipError_t collect(double ms[2], uint64_t n[2]) {
        hipError_t r = hipSuccess;
        for (int k = 0; k < 2; ++k) {
            ms[k] = 0.0;
            n[k] = ev[k].size() / 2;
            for (size_t j = 0; j + 1 < ev[k].size(); j += 2) {
                float t = 0.f;
                if (r == hipSuccess) r = hipEventElapsedTime(&t, ev[k][j], ev[k][j + 1]);
                ms[k] += t;
            }
            for (hipEvent_t e : ev[k]) (void)hipEventDestroy(e);
            ev[k].clear();
        }
        return r;
    }
    ~LaunchTimer() {
        for (auto &v : ev)
            for (hipEvent_t e : v) (void)hipEventDestroy(e);
    }
};

// The slots are split into wf_groups contiguous groups, each iterating { extend ; shade }
// on its own stream with its own queues, so one group's kernels fill the CUs that another
// group's draining launch leaves idle.  Groups never share a slot: results are unchanged.
int launch_wavefront(rt_device_scene *d, const ShardGeom &g, int spp, int depth, float *d_out, hipStream_t stream,
                     bool count, LaunchTimer &timer) {
    if (depth < 1 || depth > 15) return rt_fail(RT_ERR_LIMIT, "wavefront path: ray_depth must be in [1, 15]");
    if (spp >= (1 << 20)) return rt_fail(RT_ERR_LIMIT, "wavefront path: spp must be < 2^20");
    int rc = ensure_wf(d, g.n_pixels, depth);
    if (rc) return rc;
    rtd::WfState w = d->wf;
    w.n = g.n_pixels;
    const int G = (int)std::min<long long>(d->wf_groups, std::max<long long>(1, g.n_pixels / 4096));
    HIP_TRY(hipMemsetAsync(d->wf_count, 0, 16 * kMaxGroups, stream));
    HIP_TRY(hipMemsetAsync(d->wf_fetch, 0, sizeof(unsigned) * kParts * kMaxGroups, stream));
    HIP_TRY(hipEventRecord(d->wf_event[G], stream));
    long long lo[kMaxGroups], hi[kMaxGroups];
    bool live[kMaxGroups], dense[kMaxGroups], to_compact[kMaxGroups];
    for (int k = 0; k < G; ++k) {
        lo[k] = g.n_pixels * k / G;
        hi[k] = g.n_pixels * (k + 1) / G;
        live[k] = hi[k] > lo[k];
        dense[k] = true;   // see wf_init_kernel: dense queue until most slots are done
        to_compact[k] = false;
        HIP_TRY(hipStreamWaitEvent(d->wf_stream[k], d->wf_event[G], 0));
    }
    const long long per = (g.n_pixels + G - 1) / G;
    auto extend = count ? (d->wf_node_lds ? wf_extend_kernel<true, true> : wf_extend_kernel<true, false>)
                        : (d->wf_node_lds ? wf_extend_kernel<false, true> : wf_extend_kernel<false, false>);
    const unsigned ext_blocks = persistent_blocks(d, extend, per, d->wf_ext_bpc);
    const bool mat_lds = d->ds.n_meshes <= kMatLds;
    const unsigned sh_blocks = count ? persistent_blocks(d, wf_shade_kernel<true, true>, per)
                                     : persistent_blocks(d, wf_shade_kernel<false, true>, per);
    for (int k = 0; k < G; ++k) {
        if (!live[k]) continue;
        const unsigned init_blocks = (unsigned)std::min<long long>((hi[k] - lo[k] + 255) / 256, (long long)d->cu_count * 8);
        hipLaunchKernelGGL(wf_init_kernel, dim3(init_blocks), dim3(256), 0, d->wf_stream[k], d->ds, g, w, lo[k], hi[k],
                           d->wf_queue[0] + rtd::kQRec * lo[k], &d->wf_count[4 * k]);
    }
    HIP_TRY(hipGetLastError());
    const long long max_iter = (long long)spp * depth + 16;
    int cur = 0;
    for (long long it = 0;; ++it) {
        if (it > max_iter) return rt_fail(RT_ERR_DEVICE, "wavefront path did not drain (internal error)");
        for (int k = 0; k < G; ++k) {
            if (!live[k]) continue;
            hipStream_t sk = d->wf_stream[k];
            float4 *qi = d->wf_queue[cur] + rtd::kQRec * lo[k], *qo = d->wf_queue[1 - cur] + rtd::kQRec * lo[k];
            float4 *hits = d->wf_hits + lo[k];
            unsigned *c = &d->wf_count[4 * k];
            unsigned *fetch = &d->wf_fetch[kParts * k];
            HIP_TRY(timer.mark(0, sk));
            const unsigned npos = dense[k] ? (unsigned)(hi[k] - lo[k]) : 0u;
            hipLaunchKernelGGL(extend, dim3(ext_blocks), dim3(256), 0, sk, d->ds, qi, &c[cur], npos, hits, fetch, &c[1 - cur], d->counters, d->wf_refill, (unsigned)d->wf_chunk, d->wf_policy, d->wf_node_cost, d->wf_leaf_cost, d->wf_xcd);
            HIP_TRY(timer.mark(0, sk));
            HIP_TRY(timer.mark(1, sk));
            auto shade = count ? (mat_lds ? wf_shade_kernel<true, true> : wf_shade_kernel<true, false>)
                               : (mat_lds ? wf_shade_kernel<false, true> : wf_shade_kernel<false, false>);
            const int dense_out = dense[k] && !to_compact[k];
            hipLaunchKernelGGL(shade, dim3(sh_blocks), dim3(256), 0, sk, d->ds, g, w, spp, qi, &c[cur], npos, hits, qo, &c[1 - cur], (long long)lo[k], dense_out, fetch, d_out, d->counters);
            if (to_compact[k]) dense[k] = false;
            HIP_TRY(timer.mark(1, sk));
        }
        HIP_TRY(hipGetLastError());
        cur = 1 - cur;
        if ((it & 7) == 7) {
            for (int k = 0; k < G; ++k)
                if (live[k])
                    HIP_TRY(hipMemcpyAsync(&d->wf_host_count[k], &d->wf_count[4 * k + cur], 4, hipMemcpyDeviceToHost,
                                           d->wf_stream[k]));
            bool any = false;
            for (int k = 0; k < G; ++k) {
                if (!live[k]) continue;
                HIP_TRY(hipStreamSynchronize(d->wf_stream[k]));
                if (d->wf_host_count[k] == 0) live[k] = false;
                if (dense[k] && (double)d->wf_host_count[k] < d->wf_compact_below * (double)(hi[k] - lo[k]))
                    to_compact[k] = true;
                any = any || live[k];
            }
            if (!any) break;
        }
    }
    // the caller's stream continues after every group
    for (int k = 0; k < G; ++k) {
        HIP_TRY(hipEventRecord(d->wf_event[k], d->wf_stream[k]));
        HIP_TRY(hipStreamWaitEvent(stream, d->wf_event[k], 0));
    }
    return RT_OK;
}

int launch(rt_scene *s, const rt_params *p, float *d_out, hipStream_t stream, rt_stats *st) {
    if (!s || !p || !d_out) return rt_fail(RT_ERR_ARG, "rt_render: NULL argument");
    if (!s->dev) return rt_fail(RT_ERR_ARG, "rt_render: scene not uploaded");
    const int world = p->world > 0 ? p->world : 1, rank = p->rank, rb = p->row_block > 0 ? p->row_block : 8;
    const int spp = p->spp > 0 ? p->spp : s->samples;
    if (spp < 1) return rt_fail(RT_ERR_ARG, "rt_render: samples per pixel must be >= 1");
    if ((p->flags & RT_FLAG_FAST) && p->kernel != 0)
        return rt_fail(RT_ERR_ARG, "rt_render: fast mode (RT_FLAG_FAST) runs on kernel 0 only");
    if (p->fast_chunk < 0) return rt_fail(RT_ERR_ARG, "rt_render: fast_chunk must be >= 0");
    if ((int64_t)s->width * s->height > INT32_MAX)
        return rt_fail(RT_ERR_LIMIT, "rt_render: frames above 2^31 pixels are not supported");
    const int64_t rows = rt_shard_rows_impl(s->height, rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    ShardGeom g{s->width, rank, world, rb, (long long)rows * s->width};
    rt_device_scene *d = s->dev;
    HIP_TRY(hipSetDevice(d->device));
    const bool count = p->count != 0;
    if (count || st) HIP_TRY(hipMemsetAsync(d->counters, 0, 8 * sizeof(unsigned long long), stream));
    LaunchTimer timer;
    timer.on = st != nullptr && (p->flags & RT_FLAG_KERNEL_TIMES) != 0;
    HIP_TRY(hipMemsetAsync(d->queue, 0, 4, stream));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (st) {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, stream));
    }
    if (g.n_pixels > 0) {
        if (p->kernel == 1) {
            const unsigned blocks = (unsigned)((g.n_pixels + 255) / 256);
            if (count) hipLaunchKernelGGL(rt_pixels_kernel<true>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters);
            else hipLaunchKernelGGL(rt_pixels_kernel<false>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters);
        } else if (p->kernel == 2) {
            long long waves = (g.n_pixels + 63) / 64;
            long long want = (long long)d->cu_count * 16;
            unsigned blocks = (unsigned)((std::min(waves, want) + 3) / 4);
            if (blocks == 0) blocks = 1;
            if (count) hipLaunchKernelGGL(rt_persistent_kernel<true>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
            else hipLaunchKernelGGL(rt_persistent_kernel<false>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
        } else if (p->kernel == 4) {
            int rc = launch_wavefront(d, g, spp, s->ray_depth, d_out, stream, count, timer);
            if (rc) return rc;
        } else if (p->kernel == 0) {   // lane-resident (rt_mega.h), the default
            if (s->ray_depth < 1 || s->ray_depth > 15) return rt_fail(RT_ERR_LIMIT, "ray_depth must be in [1, 15]");
            // fast mode (RT_FLAG_FAST): work units of `cs` samples, Philox seed per sample
            const bool fast = (p->flags & RT_FLAG_FAST) != 0;
            const int cs = fast ? std::min(spp, p->fast_chunk > 0 ? p->fast_chunk : 2) : 0;
            const int chunks = fast ? (spp + cs - 1) / cs : 1;
            const long long n_items = g.n_pixels * chunks;
            if (fast && n_items > (long long)UINT32_MAX - 65536)
                return rt_fail(RT_ERR_LIMIT, "rt_render: fast mode work units exceed the 32-bit queue");
            // light-split kernel for scenes with many emissive triangles (parity mode)
            const bool lsplit = !fast && d->ds.n_lights >= d->light_split_min && d->light_split_min > 0;
            auto pick = [&](int wpe) {
                if (fast) return count ? rt_mega_kernel<true, 5, true> : rt_mega_kernel<false, 5, true>;
#if !RT_WIDE
                if (lsplit) return count ? rt_mega_kernel<true, 5, false, true> : rt_mega_kernel<false, 5, false, true>;
#endif
                switch (wpe) {
                    case 5: return count ? rt_mega_kernel<true, 5> : rt_mega_kernel<false, 5>;
                    case 6: return count ? rt_mega_kernel<true, 6> : rt_mega_kernel<false, 6>;
                    case 8: return count ? rt_mega_kernel<true, 8> : rt_mega_kernel<false, 8>;
                    default: return count ? rt_mega_kernel<true, 1> : rt_mega_kernel<false, 1>;
                }
            };
            auto mk = pick(d->mega_wpe);
            int per_cu = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mk, 256, 0));
            if (per_cu < 1) per_cu = 1;
            if (d->mega_occ > 0) per_cu = std::min(per_cu, d->mega_occ);
            const long long need = (n_items + 255) / 256, resident = (long long)d->cu_count * per_cu;
            unsigned blocks = (unsigned)std::min<long long>(need, resident);
            if (blocks == 0) blocks = 1;
            // RT_MEGA_FILL: with fewer pixels than resident lanes, launch every resident wave and
            // give each ceil(pixels / waves) lanes: more, narrower waves per SIMD
            int lane_cap = 64;
            if (d->mega_fill && need < resident && !fast) {
                blocks = (unsigned)resident;
                lane_cap = (int)std::min<long long>(64, (g.n_pixels + 4LL * blocks - 1) / (4LL * blocks));
            }
            int rc = ensure_wf(d, std::max<long long>(g.n_pixels, (long long)blocks * 256), s->ray_depth);   // vertex records
            if (rc) return rc;
            rtd::WfState w = d->wf;
            w.n = g.n_pixels;
            w.lanes = (long long)blocks * 256;   // LaneRec slots (<= the workspace capacity)
            // pixel order, from the per-pixel costs of the last counting render of this shard
            // (results never depend on it):
            //   * heaviest first, so the frame's tail is made of cheap pixels;
            //   * spread (RT_MEGA_SPREAD, default): the first claims, one pixel per lane, give
            //     every wave one pixel of each cost stratum.  A pixel's 256 samples are one
            //     sequential chain, and with ~1 pixel per lane (8 GPUs) the frame is the
            //     heaviest pixel's chain; with light wave-mates that finish early, it runs in a
            //     sparse wave (fewer divergent paths per iteration, shading batches not held
            //     back).  Rank-0 shard of an 8-way split: 490 -> 353 ms; 1 GPU: +1-2%.
            //     Plain heaviest-first (RT_MEGA_SPREAD=0) only with >= RT_MEGA_ORDER_MIN pixels
            //     per lane: with fewer it clusters the heavy pixels in the same waves.
            const bool many = !fast && (g.n_pixels >= (long long)d->mega_order_min * blocks * 256 || d->mega_spread);
            const bool same = many && d->order && d->order_n == g.n_pixels && d->order_key[0] == rank &&
                              d->order_key[1] == world && d->order_key[2] == rb && d->order_valid && d->mega_reorder;
            unsigned *cost = nullptr;
            if (count && st && d->mega_reorder && many) {
                if (d->order_cap < g.n_pixels) {
                    if (d->order) (void)hipFree(d->order);
                    if (d->order_cost) (void)hipFree(d->order_cost);
                    d->order = nullptr;
                    d->order_cost = nullptr;
                    d->order_cap = 0;
                    HIP_TRY(hipMalloc((void **)&d->order, sizeof(int) * g.n_pixels));
                    HIP_TRY(hipMalloc((void **)&d->order_cost, sizeof(unsigned) * g.n_pixels));
                    d->order_cap = g.n_pixels;
                }
                cost = d->order_cost;
            }
            float *k_out = d_out;
            if (fast) {
                if (d->fast_part_cap < n_items * 3) {
                    if (d->fast_part) (void)hipFree(d->fast_part);
                    d->fast_part = nullptr;
                    d->fast_part_cap = 0;
                    HIP_TRY(hipMalloc((void **)&d->fast_part, sizeof(float) * n_items * 3));
                    d->fast_part_cap = n_items * 3;
                }
                k_out = d->fast_part;
            }
            if (d->mega_times && d->mega_tfin_n < g.n_pixels) {   // RT_MEGA_TIMES: per-pixel finish clocks
                if (d->mega_tfin) (void)hipFree(d->mega_tfin);
                HIP_TRY(hipMalloc((void **)&d->mega_tfin, sizeof(unsigned long long) * g.n_pixels));
                d->mega_tfin_n = g.n_pixels;
            }
            unsigned long long t_launch = 0;
            if (d->mega_times) {
                HIP_TRY(hipStreamSynchronize(stream));
                t_launch = 0;
            }
#ifdef RT_MEGA_PROF
            {
                const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mega_prof), z, sizeof z, 0, hipMemcpyHostToDevice, stream));
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mega_seg), z, sizeof z, 0, hipMemcpyHostToDevice, stream));
            }
#endif
            hipLaunchKernelGGL(mk, dim3(blocks), dim3(256), 0, stream, d->ds, g, w, spp, k_out, d->counters, d->queue,
                               d->mega_shade_min | d->mega_trav_min << 8 | (lane_cap & 127) << 16 |
                                   (d->mega_team ? 1 << 23 : 0),
                               same ? (const int *)d->order : nullptr, cost,
                               d->mega_times && !fast ? d->mega_tfin : nullptr, cs);
            HIP_TRY(hipGetLastError());
            if (fast) {
                const long long n3 = g.n_pixels * 3;
                hipLaunchKernelGGL(rt_fast_reduce_kernel, dim3((unsigned)((n3 + 255) / 256)), dim3(256), 0, stream,
                                   (const float *)d->fast_part, d_out, n3, chunks);
                HIP_TRY(hipGetLastError());
            }
#ifdef RT_MEGA_PROF
            {
                unsigned long long pf[8];
                HIP_TRY(hipMemcpyFromSymbolAsync(pf, HIP_SYMBOL(g_mega_prof), sizeof pf, 0, hipMemcpyDeviceToHost, stream));
                HIP_TRY(hipStreamSynchronize(stream));
                const double tot = (double)(pf[0] + pf[1] + pf[2]);
                std::fprintf(stderr,
                             "[mega prof] count=%d waves=%llu cycles/wave=%.3g shade=%.3f trav=%.3f assign=%.3f "
                             "shade_iters/wave=%.0f trav_iters/wave=%.0f ready/shade=%.1f trav_lanes/iter=%.1f "
                             "cyc/shade_iter=%.0f cyc/trav_iter=%.0f\n",
                             (int)count, pf[7], tot / pf[7], pf[0] / tot, pf[1] / tot, pf[2] / tot,
                             (double)pf[3] / pf[7], (double)pf[4] / pf[7], (double)pf[5] / pf[3],
                             (double)pf[6] / pf[4], (double)pf[0] / pf[3], (double)pf[1] / pf[4]);
                unsigned long long sg[8];
                HIP_TRY(hipMemcpyFromSymbolAsync(sg, HIP_SYMBOL(g_mega_seg), sizeof sg, 0, hipMemcpyDeviceToHost, stream));
                HIP_TRY(hipStreamSynchronize(stream));
                std::fprintf(stderr, "[mega prof] shade segments, cycles per shade iteration: mesh+emission=%.0f "
                             "normal=%.0f mr=%.0f sample=%.0f pdf=%.0f base+brdf=%.0f; team rays/wave=%.1f cyc/team ray=%.0f\n",
                             (double)sg[0] / pf[3], (double)sg[1] / pf[3], (double)sg[2] / pf[3],
                             (double)sg[3] / pf[3], (double)sg[4] / pf[3], (double)sg[5] / pf[3],
                             (double)sg[7] / pf[7], sg[7] ? (double)sg[6] / sg[7] : 0.0);
            }
#endif
            if (d->mega_times && count) {   // print finish-time percentiles (ms after the first finish) to stderr
                std::vector<unsigned long long> t(g.n_pixels);
                HIP_TRY(hipMemcpyAsync(t.data(), d->mega_tfin, sizeof(unsigned long long) * g.n_pixels,
                                       hipMemcpyDeviceToHost, stream));
                HIP_TRY(hipStreamSynchronize(stream));
                std::sort(t.begin(), t.end());
                int rate_khz = 0;
                (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, d->device);
                const double to_ms = rate_khz > 0 ? 1.0 / rate_khz : 1e-5;
                std::fprintf(stderr, "[mega times] n=%lld wall-clock kHz=%d finish ms:", (long long)g.n_pixels, rate_khz);
                for (double q : {0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99, 0.999, 1.0}) {
                    const size_t k = std::min(t.size() - 1, (size_t)(q * (t.size() - 1)));
                    std::fprintf(stderr, " p%g=%.1f", q * 100, (double)(t[k] - t[0]) * to_ms);
                }
                std::fprintf(stderr, "\n");
                (void)t_launch;
            }
            if (cost) {   // build the order for the next renders of this shard
                std::vector<unsigned> c(g.n_pixels);
                HIP_TRY(hipMemcpyAsync(c.data(), cost, sizeof(unsigned) * g.n_pixels, hipMemcpyDeviceToHost, stream));
                HIP_TRY(hipStreamSynchronize(stream));
                std::vector<int> ord(g.n_pixels);
                for (long long k = 0; k < g.n_pixels; ++k) ord[k] = (int)k;
                if (d->mega_tile > 0) {
                    // tiles of T x T shard pixels, heaviest tile first, scanline order inside
                    // a tile (neighbouring queue entries stay neighbouring pixels)
                    const int T = d->mega_tile, tw = (g.width + T - 1) / T;
                    const long long rows = g.n_pixels / g.width;
                    std::vector<unsigned long long> tc((size_t)tw * ((rows + T - 1) / T), 0);
                    auto tile = [&](int p) { return (size_t)((p / g.width) / T) * tw + (p % g.width) / T; };
                    for (long long k = 0; k < g.n_pixels; ++k) tc[tile((int)k)] += c[k];
                    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
                        const size_t ta = tile(a), tb = tile(b);
                        if (ta == tb) return false;
                        return tc[ta] != tc[tb] ? tc[ta] > tc[tb] : ta < tb;
                    });
                } else {
                    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return c[a] > c[b]; });
                }
                if (d->mega_spread) {
                    // the first claims (one per lane: every wave takes lane_cap consecutive queue
                    // entries at its start) get the heaviest pixels, but each wave one pixel of
                    // every cost stratum, so a heavy pixel's wave-mates are light and finish early;
                    // later claims stay heaviest-first
                    const long long groups = 4LL * blocks, first = std::min<long long>(g.n_pixels, groups * lane_cap);
                    std::vector<int> sp(ord);
                    long long r = 0;
                    for (long long j = 0; j < lane_cap; ++j)
                        for (long long gi = 0; gi < groups; ++gi) {
                            const long long q = gi * lane_cap + j;
                            if (q < first) sp[q] = ord[r++];
                        }
                    ord.swap(sp);
                }
                HIP_TRY(hipMemcpy(d->order, ord.data(), sizeof(int) * g.n_pixels, hipMemcpyHostToDevice));
                d->order_n = g.n_pixels;
                d->order_key[0] = rank;
                d->order_key[1] = world;
                d->order_key[2] = rb;
                d->order_valid = true;
            }
        } else {
            // persistent wave kernel: exactly the resident blocks (occupancy query), capped by the work
            int per_cu = 0;
            if (count) HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rt_wave_kernel<true>, 256, 0));
            else HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rt_wave_kernel<false>, 256, 0));
            if (per_cu < 1) per_cu = 1;
            long long need = (g.n_pixels + 255) / 256;
            unsigned blocks = (unsigned)std::min<long long>(need, (long long)d->cu_count * per_cu);
            if (blocks == 0) blocks = 1;
            if (count) hipLaunchKernelGGL(rt_wave_kernel<true>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
            else hipLaunchKernelGGL(rt_wave_kernel<false>, dim3(blocks), dim3(256), 0, stream, d->ds, g, spp, d_out, d->counters, d->queue);
        }
        HIP_TRY(hipGetLastError());
    }
    if (st) {
        HIP_TRY(hipEventRecord(e1, stream));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        std::memset(st, 0, sizeof *st);
        st->pixels = (uint64_t)g.n_pixels;
        st->samples = (uint64_t)g.n_pixels * (uint64_t)spp;
        st->render_ms = ms;
        double kms[2];
        uint64_t kn[2];
        HIP_TRY(timer.collect(kms, kn));
        st->extend_ms = kms[0];
        st->shade_ms = kms[1];
        st->extend_launches = kn[0];
        st->shade_launches = kn[1];
        unsigned long long c[8];
        HIP_TRY(hipMemcpy(c, d->counters, sizeof c, hipMemcpyDeviceToHost));
        st->extend_rays = c[7];
        if (count) {
            st->rays = c[0]; st->aabb_tests = c[1]; st->tri_tests = c[2];
            st->light_queries = c[3]; st->light_aabb_tests = c[4]; st->light_tri_tests = c[5];
            st->shading_hits = c[6];
        }
    }
    return RT_OK;
}

}  // namespace

void rt_device_scene_release(rt_scene *s) {
    if (!s || !s->dev) return;
    rt_device_scene *d = s->dev;
    if (hipSetDevice(d->device) == hipSuccess) {
        if (d->buf) (void)hipFree(d->buf);
        if (d->counters) (void)hipFree(d->counters);
        if (d->queue) (void)hipFree(d->queue);
        if (d->wf_buf) (void)hipFree(d->wf_buf);
        if (d->wf_count) (void)hipFree(d->wf_count);
        if (d->wf_fetch) (void)hipFree(d->wf_fetch);
        if (d->order) (void)hipFree(d->order);
        if (d->order_cost) (void)hipFree(d->order_cost);
        if (d->mega_tfin) (void)hipFree(d->mega_tfin);
        if (d->fast_part) (void)hipFree(d->fast_part);
        if (d->wf_host_count) (void)hipHostFree(d->wf_host_count);
        for (hipStream_t &x : d->wf_stream)
            if (x) (void)hipStreamDestroy(x);
        for (hipEvent_t &x : d->wf_event)
            if (x) (void)hipEventDestroy(x);
    }
    delete d;
    s->dev = nullptr;
}

extern "C" {

int rt_scene_upload(rt_scene *s, int32_t device) {
    if (!s) return rt_fail(RT_ERR_ARG, "rt_scene_upload: NULL scene");
    return ensure_device_scene(s, device);
}

int rt_render_device(rt_scene *s, const rt_params *p, float *d_out, void *stream, rt_stats *st) {
    return launch(s, p, d_out, (hipStream_t)stream, st);
}

int rt_tonemap_u8_device(const float *d_sum, int32_t width, int32_t height, int32_t spp, uint8_t *d_rgb, void *stream) {
    if (!d_sum || !d_rgb || width <= 0 || height <= 0 || spp <= 0)
        return rt_fail(RT_ERR_ARG, "rt_tonemap_u8_device: bad argument");
    static bool uploaded[64] = {false};
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return rt_fail(RT_ERR_DEVICE, "rt_tonemap_u8_device: device id");
    if (!uploaded[dev]) {
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(k_quant_thr), rtm::kQuantThr, sizeof rtm::kQuantThr));
        uploaded[dev] = true;
    }
    const long long n = (long long)width * height * 3;
    const unsigned blocks = (unsigned)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(rt_finish_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_sum, n,
                       1.f / (float)spp, d_rgb);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_render(rt_scene *s, const rt_params *p, float *out, rt_stats *st) {
    if (!s || !p || !out) return rt_fail(RT_ERR_ARG, "rt_render: NULL argument");
    if (!s->dev) {
        int rc = ensure_device_scene(s, 0);
        if (rc) return rc;
    }
    const int world = p->world > 0 ? p->world : 1, rb = p->row_block > 0 ? p->row_block : 8;
    const int64_t rows = rt_shard_rows_impl(s->height, p->rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    const size_t bytes = (size_t)rows * s->width * 3 * sizeof(float);
    HIP_TRY(hipSetDevice(s->dev->device));
    float *d_out = nullptr;
    HIP_TRY(hipMalloc(&d_out, bytes ? bytes : 4));
    rt_stats local;
    int rc = launch(s, p, d_out, nullptr, st ? st : &local);
    if (rc == RT_OK) {
        hipError_t e = hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = rt_fail(RT_ERR_DEVICE, std::string("rt_render copy: ") + hipGetErrorString(e));
    }
    (void)hipFree(d_out);
    return rc;
}

int rt_intersect_rays(rt_scene *s, int64_t n, const float *org, const float *dir, float *out_f, int64_t *out_i) {
    if (!s || n < 0 || (n > 0 && (!org || !dir || !out_f || !out_i))) return rt_fail(RT_ERR_ARG, "rt_intersect_rays: bad argument");
    if (n == 0) return RT_OK;
    if (!s->dev) {
        int rc = ensure_device_scene(s, 0);
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(s->dev->device));
    float *d_o = nullptr, *d_d = nullptr, *d_f = nullptr;
    long long *d_i = nullptr;
    const size_t v3 = (size_t)n * 3 * sizeof(float);
    hipError_t e = hipMalloc(&d_o, v3);
    if (e == hipSuccess) e = hipMalloc(&d_d, v3);
    if (e == hipSuccess) e = hipMalloc(&d_f, (size_t)n * 4 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_i, (size_t)n * 6 * sizeof(long long));
    if (e == hipSuccess) e = hipMemcpy(d_o, org, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dir, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rt_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, s->dev->ds, (long long)n,
                           d_o, d_d, d_f, d_i);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_f, d_f, (size_t)n * 4 * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_i, d_i, (size_t)n * 6 * sizeof(long long), hipMemcpyDeviceToHost);
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_f);
    (void)hipFree(d_i);
    if (e != hipSuccess) return rt_fail(RT_ERR_DEVICE, std::string("rt_intersect_rays: ") + hipGetErrorString(e));
    return RT_OK;
}

#if defined(RT_DEBUG_CHECKS)
// debug builds only: first recorded index violation (code << 56 | value), 0 = none
int rt_debug_take(unsigned long long *word) {
    unsigned long long z = 0;
    HIP_TRY(hipMemcpyFromSymbol(word, HIP_SYMBOL(rt_debug_word), sizeof z));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rt_debug_word), &z, sizeof z));
    return RT_OK;
}
#endif

// rt_device_selfcheck 0: rcp_ieee against the IEEE division 1.f / x over every float x
// with a normal reciprocal path (|x| in [2^-126, 2^125)), on the device.
__global__ void __launch_bounds__(256) rcp_check_kernel(unsigned long long *bad) {
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)i);
        const float ax = fabsf(x);
        if (!(ax >= 0x1p-126f && ax < 0x1p125f)) continue;
        const float a = rtd::rcp_ieee(x), b = 1.f / x;
        local += __float_as_uint(a) != __float_as_uint(b);
    }
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(bad, local);
}

int rt_device_selfcheck(int32_t which, uint64_t *mismatches) {
    if (!mismatches) return rt_fail(RT_ERR_ARG, "rt_device_selfcheck: null output");
    if (which != 0) return rt_fail(RT_ERR_ARG, "rt_device_selfcheck: unknown check " + std::to_string(which));
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, sizeof *d));
    hipError_t e = hipMemset(d, 0, sizeof *d);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rcp_check_kernel, dim3(4096), dim3(256), 0, nullptr, d);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return rt_fail(RT_ERR_DEVICE, std::string("rt_device_selfcheck: ") + hipGetErrorString(e));
    *mismatches = h;
    return RT_OK;
}

int32_t rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_device_synchronize(void) {
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

}  // extern "C"

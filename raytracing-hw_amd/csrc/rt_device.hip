// rt_device.hip — MI355X (gfx950) render kernels and the device half of the C ABI.
//
// Kernels (the per-pixel sample loop of Scene::render, scene.cpp:31-52, and its finish):
//   rt_mega_kernel          lane-resident persistent path tracer (rt_mega.h), the default:
//                           every lane runs whole pixels, traversal one unit per iteration,
//                           shading batched per wave; also fast mode (RT_FLAG_FAST) and the
//                           counting pre-pass that orders pixels heaviest-first
//   wf_{init,extend,shade}  wavefront schedule of the same arithmetic (kernel 4, rt_wavefront.h)
//   rt_finish_kernel        mean -> ACES -> gamma -> 8-bit (scene.cpp:54-64)
//   rt_rays_kernel          BVH::intersect + light pdf for explicit rays (test entry)
// Every schedule writes the per-pixel float RGB sum (sample_canvas, scene.cpp:20,42) of the
// owned rows; the bits do not depend on the kernel, the launch shape, the pixel order or the
// partition.
//
// Concurrency: one render per (scene, device) may be in flight at a time (the pixel queue,
// counters, vertex records and order buffers of a device copy are shared by its launches);
// renders of the same scene on different devices are independent (rt_render_multi).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt_path.h"
#include "rt_wavefront.h"
#include <type_traits>
#include "rt_mega.h"
#include "rt_quant_lut.h"
#include "rt_scene.h"
#include "rt_bvh_layout.h"

using rtd::Counters;
using rtd::DevScene;
using rtd::ShardGeom;
using rtd::shard_row;

// Tuned constants of the default kernel (measured values in DESIGN.md §5-6).
#ifndef RT_MEGA_WPE
#define RT_MEGA_WPE 5
#endif
constexpr int kMegaWpe = RT_MEGA_WPE;   // waves per SIMD the register allocation targets (96 VGPRs)
// The runahead instantiation runs shards of at most kSpecPixelsPerLane (2) pixels per lane
// (an 8-way shard of the headline: 1013 blocks, 4 waves per SIMD, one pixel per lane; a
// 4-way shard two): 128 VGPRs instead of 96 keep its management pass from spilling the loop.
#ifndef RT_SPEC_WPE
#define RT_SPEC_WPE 4
#endif
constexpr int kMegaWpeSpec = RT_SPEC_WPE;
#ifndef RT_SHADE_MIN
#define RT_SHADE_MIN 48
#endif
// The runahead kernel (4- and 8-way shards) shades at 40 READY lanes: its waves thin out
// early, and a heavy chain's lane waits less for its batch than at the plain kernel's 48.
// Round 3 (window 3): slowest 8-way shard 207.5-207.7 ms at 40 against 208.6-211.7 at 32 and
// 214.8 at 24, 4-way 346-347 vs 352-354 (profiles/r03_ab.jsonl r03ah, r03ai).  Round 2: 294 ms
// at 32 against 297-299 at 48 (profiles/r02_tail_ab.jsonl).
// Round 5, with the runahead priority (rt_mega.h RT_SPEC_PRIO): 48 READY lanes, 8-way shards
// 187.2 max / 185.6 mean ms against 188.2-188.5 / 186.9-187.5 at 40 (profiles/r05f_prio_variants_ab.jsonl).
// Round 6, with leaf deferral (rt_wavefront.h RT_LEAF_DEFER): 44 READY lanes, 12 coop leaf
// records and at most 4 deferrals in a row, slowest 8-way shard 174.4-175.8 / mean 173.2-173.7
// ms against 176.1-176.5 / 174.4-174.9 at 48, 16 and 3 (profiles/r06w_spec_tuning_ab.jsonl,
// three runs each; 52 lanes 179.6-179.8 in r06v).
#ifndef RT_SPEC_SHADE_MIN
#define RT_SPEC_SHADE_MIN 44
#endif
constexpr int kSpecShadeMin = RT_SPEC_SHADE_MIN;   // the runahead kernel's batch threshold
constexpr int kShadeMin = RT_SHADE_MIN;   // a wave shades once this many lanes are READY (or none traverses)
// RT_PACK_TRAV: through a shading pass, a lane that does not shade holds its traversal phase,
// stack depth and state packed in one register (the loop body below).  With RT_TID_REMAT
// (rt_mega.h) the plain kernel spills 16 VGPRs instead of 33 and writes 0.11 instead of
// 0.37 TB per frame (WRITE_SIZE: 53 instead of 178 B per ray); frame 1038-1041 ms against
// 1093-1094 (profiles/r05n_ab.jsonl).  0: A/B.
#ifndef RT_PACK_TRAV
#define RT_PACK_TRAV 1
#endif
constexpr bool kPackTrav = RT_PACK_TRAV != 0;
#ifndef RT_INV_RECOMPUTE
#define RT_INV_RECOMPUTE 1
#endif
constexpr bool kInvRecompute = RT_INV_RECOMPUTE != 0;
// Traversal iterations between two shading passes run as an inner loop of their own (no pixel
// claim, runahead pass or schedule decision per iteration), one cooperative step each
// (rt_wavefront.h trav_step_coop: leaf work spread over the wave).  The lane-resident
// kernel's traversal state shares the node and leaf fields (rt_wavefront.h TravStateU; the
// runahead kernel keeps TravState).
// Leaf lanes a coop step serves (32 B of LDS per wave each).  The plain kernel's block is at
// 30 KB and must stay within 32 KB minus what the runtime keeps, for 5 blocks per CU: 16
// records (32 KB) measured 1426 ms against 1272 at 8 (4 blocks per CU).  The runahead kernel
// runs 4 blocks per CU anyway (128 VGPRs): 16 there (8-way slowest shard 245 vs 249 ms).
#ifndef RT_COOP_LEAVES
#define RT_COOP_LEAVES 8
#endif
constexpr int kCoopLeavesPlain = RT_COOP_LEAVES;
#ifndef RT_SPEC_COOP_LEAVES
#define RT_SPEC_COOP_LEAVES 12   // (16 until round 6's leaf deferral: see RT_SPEC_SHADE_MIN)
#endif
constexpr int kCoopLeavesSpec = RT_SPEC_COOP_LEAVES;   // the runahead kernel's coop leaf records per wave
// The runahead kernel's coop step issues the child-pair loads from node lanes only
// (rt_wavefront.h trav_step_coop MASK_LOAD; the plain kernel measured slower with it).
#ifndef RT_SPEC_MASK_LOAD
#define RT_SPEC_MASK_LOAD 1
#endif
constexpr bool kSpecMaskLoad = RT_SPEC_MASK_LOAD != 0;
// Leaf rounds per coop step (rt_wavefront.h trav_step_coop round_min): a further round
// while at least this many leaf lanes are unserved.  Plain kernel: 8 (sponza 1080p 1292 ->
// 1278 ms against one round per step).  Runahead kernel: 4 on scenes of fewer than
// kCoopRoundNodes BVH nodes, where most traversal steps are leaf steps (cornell 512x512x64,
// 36 triangles: 26.8 -> 16.7 ms), one round per step on larger ones (the 8-way sponza
// shards: 1% slower with rounds) (profiles/r03_ab.jsonl r03q-s).
#ifndef RT_COOP_ROUND_MIN
#define RT_COOP_ROUND_MIN 8
#endif
#ifndef RT_SPEC_COOP_ROUND_MIN
#define RT_SPEC_COOP_ROUND_MIN 4
#endif
constexpr int kCoopRoundMinPlain = RT_COOP_ROUND_MIN;
constexpr int kCoopRoundMinSpec = RT_SPEC_COOP_ROUND_MIN;   // small scenes
constexpr int kCoopRoundNodes = 4096;
// Pixel order pre-pass (launch_order).  Compile-time only, for A/B builds (make variant).
// Measured on sponza 1080p x256spp (tools/order_ab.py, profiles/r02_order_ab.jsonl): 1 spp and
// a 9 x 9 box filter (1399 ms, pre-pass 6.8 ms) against row-major order (1436 ms), 2 spp
// unfiltered (1470 ms: a noisy order loses the coherence of row-major order and gains
// nothing), 2 spp 5 x 5 (1407 ms), 8 spp 3 x 3 (1429 ms); 8-way shards, slowest of the 8:
// 346 ms against 478 ms in row-major order.  Ordering 64-pixel runs instead of pixels keeps
// rows coherent but loses the spread (8-way 476 ms).
#ifndef RT_ORDER_SPP
#define RT_ORDER_SPP 1
#endif
#ifndef RT_ORDER_RADIUS
#define RT_ORDER_RADIUS 4
#endif
constexpr int kOrderSpp = RT_ORDER_SPP;       // samples per pixel of the counting pre-pass
constexpr int kOrderRadius = RT_ORDER_RADIUS;  // box filter of the pre-pass costs ((2r+1)^2 pixels)
// The pre-pass and sort cost about one sample per pixel, so below kOrderMinSpp the order
// is not built unless asked for (RT_FLAG_HEAVY_ORDER): row-major measured faster there
// (profiles/r02_configs.jsonl: C1 256x256x4 4.5 vs 5.0 ms, C2 512x512x64 17.7 vs 18.0 ms, C5
// 3840x2160 at 16 spp 378 vs 397 ms; at 256 spp the order wins, C3 748 vs 779 ms, headline
// 1357 vs 1393 ms).
constexpr int kOrderMinSpp = 128;
constexpr int kFastMaxChunks = 128;  // fast mode: at most this many work units per pixel
// Round 3 (runahead window 3): up to 2 pixels per lane, so the 4-way shards of the headline
// (2 per lane) use it too: slowest 4-way shard 347.5 vs 358.7 ms; at 4 per lane (2-way)
// 636 vs 625 (profiles/r03_ab.jsonl r03ah24).
#ifndef RT_SPEC_PIXELS_PER_LANE
#define RT_SPEC_PIXELS_PER_LANE 2
#endif
constexpr long long kSpecPixelsPerLane = RT_SPEC_PIXELS_PER_LANE;   // runahead kernel up to this many pixels per lane
// Hand-off (round 6): a parity render on the plain kernel (more than kSpecPixelsPerLane pixels
// per lane) ends its tail in the runahead kernel.  A plain wave whose queue is empty parks its
// pixels once fewer than kHandoffBelow of its lanes hold one (each at its next sample end, with
// its RNG state and sum), and a runahead launch over the whole resident grid resumes them
// (kHandoffPct percent dealt at its start, the rest claimed in the tail): the plain kernel's
// sparse tail waves, where most lanes idle while a few pixels finish their chains, become
// runahead records.  Headline frame 1048.3 vs 1061.5 ms on one box, 2-way shards 578.6 vs
// 580.6 ms, same bits; parking at 48 / 60 held pixels 1049.0 / 1050.8 ms, 70% dealt 1050.2 ms
// (profiles/r06g_handoff_ab.jsonl).  RT_FLAG_NO_RUNAHEAD turns it off with the runahead.
#ifndef RT_HANDOFF_BELOW
#define RT_HANDOFF_BELOW 56
#endif
#ifndef RT_HANDOFF_PCT
#define RT_HANDOFF_PCT 100
#endif
// RT_HANDOFF_SPREAD: the runahead launch deals the parked pixels with the most work left
// ((samples left) x (pre-pass estimate)) one per wave, instead of in park-list slot order,
// where a plain wave's consecutive claims (the last pixels of the order, those that end the
// frame) sit together and share one wave's idle lanes.
#ifndef RT_HANDOFF_SPREAD
#define RT_HANDOFF_SPREAD 1
#endif
constexpr int kHandoffBelow = RT_HANDOFF_BELOW;
constexpr int kHandoffPct = RT_HANDOFF_PCT;
constexpr bool kHandoffSpread = RT_HANDOFF_SPREAD != 0;
// Diagnostics (A/B builds only): only every k-th lane of a wave claims pixels, so a wave
// holds at most 64 / k pixels and the grid grows k-fold (lockstep study).
#ifndef RT_CLAIM_STRIDE
#define RT_CLAIM_STRIDE 1
#endif
constexpr int kClaimStride = RT_CLAIM_STRIDE;
constexpr int kWfRefill = 8;         // wavefront extend: idle lanes before a wave refills
constexpr unsigned kWfChunk = 64;    // wavefront extend: queue entries claimed per atomic
constexpr double kWfCompactBelow = 0.75;   // wavefront: dense queue until this active fraction

// The device image of a scene (built once on the host, copied to every device it renders on).
struct rt_device_blob {
    std::vector<uint8_t> bytes;
    size_t o_tri, o_attr, o_tan, o_node, o_light, o_lnode, o_mf, o_mt, o_nt, o_ti, o_tx, o_lut;
};

struct rt_device_scene {
    int device = -1;
    void *buf = nullptr;               // one allocation holding every scene array
    DevScene ds{};
    unsigned long long *counters = nullptr;  // 16 x u64: [0, 8) the render, [8, 16) the order pre-pass
    unsigned long long *queue = nullptr;     // 8 x u64: work counters of the render and the pre-pass, the
                                             // hand-off's park count (u32), its runahead launch's claims and
                                             // the address of its park list (rt_mega_kernel `mode`)
    int cu_count = 0;
    // vertex records (lane-resident) / path state and queues (wavefront)
    void *wf_buf = nullptr;
    long long wf_cap = 0;
    int wf_D = 0;
    rtd::WfState wf{};
    float4 *wf_queue[2] = {nullptr, nullptr};
    float4 *wf_hits = nullptr;
    unsigned *wf_count = nullptr;       // [0], [1]: queue counts (active rays)
    unsigned *wf_fetch = nullptr;       // extend claim counter
    unsigned *wf_host_count = nullptr;  // pinned
    float *fast_part = nullptr;         // fast mode / pre-pass: work-unit partial sums
    size_t fast_part_bytes = 0;
    // pixel order of the current render (heaviest first, spread; see launch_order)
    void *order_buf = nullptr;
    size_t order_bytes = 0;
    // rt_render_frame, kept between frames: the device's render and copy streams, two shard
    // buffers (float sums then 8-bit rows) and the events that order their reuse; on the root
    // device also the staging / frame buffers and the row map (FrameRoot)
    hipStream_t fr_stream = nullptr, cp_stream = nullptr;
    void *fr_buf[2] = {nullptr, nullptr};
    size_t fr_bytes[2] = {0, 0};
    hipEvent_t fr_copied[2] = {nullptr, nullptr};   // copy of buffer b done (reuse after it)
    hipEvent_t fr_finished = nullptr;               // shard finished to 8 bits (copy may start)
    hipEvent_t fr_last = nullptr;                   // the device's last copy of the frame done
    void *root_buf = nullptr;
    size_t root_bytes = 0;
};

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return rt_fail(RT_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

namespace {

// Restores the calling thread's current HIP device on every return path.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// HIP events released on every return path.
struct EventSet {
    std::vector<hipEvent_t> ev;
    hipError_t make(hipEvent_t &e) {
        hipError_t r = hipEventCreate(&e);
        if (r == hipSuccess) ev.push_back(e);
        return r;
    }
    ~EventSet() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
};

// Device buffer that only grows (contents not kept).
hipError_t grow(void **p, size_t *cap, size_t need) {
    if (*p && *cap >= need) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, need ? need : 256);
    if (e == hipSuccess) *cap = need;
    return e;
}

}  // namespace

// ------------------------------------------------------------------------ kernels
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

// ------------------------------------------------------------------------ lane-resident (kernel 0)
// rt_mega.h: every lane runs whole pixels; traversal one unit per iteration, shading batched
// per wave (READY lanes wait for kShadeMin of them or for no lane left traversing).
#ifdef RT_MEGA_PROF
// Diagnostics build (make prof): per-wave clock64() split of the main loop.
// [0] shade-iteration cycles [1] traversal-iteration cycles [2] pixel-assign cycles
// [3] shade iterations [4] traversal iterations [5] sum of ready lanes over shade iterations
// [6] sum of traversing lanes over traversal iterations [7] waves
__device__ unsigned long long g_mega_prof[8];
__device__ unsigned long long g_mega_seg[8];   // shading segments (rt_path.h RT_PROF_SEG)
// per-wave start and end (wall_clock64, 100 MHz): the distribution of wave finish times
constexpr int kProfWaves = 16384;
__device__ unsigned long long g_wave_t[2 * kProfWaves];
__device__ unsigned int g_wave_n;
// time buckets of 5 ms (wall clock since the wave's start; the waves of a launch start within
// microseconds of each other): [0] traversal iterations [1] traversing lanes summed over them
// [2] lanes holding work (state != idle) summed over them [3] shading passes [4] READY lanes
// summed over them [5] management passes (runahead kernel)
constexpr int kTb = 256, kTbN = 6;
constexpr unsigned long long kTbTicks = 500000;   // 5 ms at 100 MHz
__device__ unsigned long long g_tb[kTb * kTbN];
struct TbAcc {
    int b = 0;
    unsigned long long c[kTbN] = {0, 0, 0, 0, 0, 0};
    __device__ void at(unsigned long long t0) {   // (every lane; lane 0 flushes)
        const unsigned long long e = (wall_clock64() - t0) / kTbTicks;
        const int nb = e < (unsigned long long)kTb ? (int)e : kTb - 1;
        if (nb != b) flush(nb);
    }
    __device__ void flush(int nb) {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < kTbN; ++k)
                if (c[k]) atomicAdd(&g_tb[b * kTbN + k], c[k]);
        for (int k = 0; k < kTbN; ++k) c[k] = 0;
        b = nb;
    }
};
#endif
// FAST (RT_FLAG_FAST): queue items are (chunk, pixel) work units of `cs`
// samples with per-sample Philox seeds; `out` is then the chunk-major partial buffer that
// rt_fast_reduce_kernel folds.  LSPLIT (RT_FLAG_LIGHT_SPLIT, §8(f)3): the light pdf's
// light-BVH walk as a lane state (rt_mega.h light_step).  `order` (parity mode): queue item
// p renders shard pixel order[p].  `cost` (COUNT only): per-pixel traversal tests out.
// Exit: the queue is monotonic, so once a claim reaches n_items a wave stops claiming; the
// loop ends when no lane of the wave holds work, so the grid always drains.
// SPEC (parity renders without counting): a wave whose claim finds the queue empty enters its
// tail and runs speculative sample runahead (rt_mega.h spec_manage) on its idle lanes.  A
// separate instantiation, so the kernel without it keeps its own register allocation.
// `mode` (0 for the default schedules) packs the hand-off's settings (one kernel argument: the
// kernel is short of SGPRs, which spill into VGPRs):
//   bits 0-7   park_below > 0 (plain kernel): a wave whose queue is empty and that holds fewer
//              than park_below pixels parks them, each at its next sample end, in the park list
//              at its lane slot (rt_mega.h park_pixel; the list's address in queue[4], read where
//              used: no register held in the loop);
//   bits 8-15  resume_pct > 0 (SPEC): the items are that park list's slots (st.n of them); wave
//              w of the grid takes slots [w * per, (w + 1) * per), its lanes below per one each
//              (per: resume_pct percent of the slots over the grid's waves, at most 64), skips
//              the empty ones and enters its tail at once; the slots past the grid's share are
//              claimed in the tail (rt_mega.h SpecClaim) through the counter at queue + 3.
template <bool COUNT, bool FAST = false, bool LSPLIT = false, bool SPEC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SPEC ? kMegaWpeSpec : kMegaWpe, 8)))
rt_mega_kernel(DevScene sc_in, ShardGeom g, rtd::WfState st, int spp, float *out, unsigned long long *counters,
               unsigned long long *queue, const int *order, unsigned *cost, int cs, int mode) {
    constexpr bool kSpec = SPEC && !COUNT && !FAST && !LSPLIT;
    const int park_below = mode & 255, resume_pct = (mode >> 8) & 255;
    const uint4 *resume = kSpec && resume_pct > 0 ? (const uint4 *)queue[4] : nullptr;
    const long long n_items = FAST ? g.n_pixels * (long long)((spp + cs - 1) / cs) : (kSpec && resume) ? st.n : g.n_pixels;
    const int lane = threadIdx.x & 63;
    // sRGB texel-decode table in LDS: the shading's lane-dependent lookups become ds_reads (the
    // linear decode is computed: rt_path.h texel_decode)
    __shared__ float lut[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) lut[k] = sc_in.lut[k];
    __syncthreads();
    DevScene sc = sc_in;
    sc.lut = lut;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    constexpr int kK = kSpec ? rtd::kLdsStackSpec : rtd::kLdsStack;   // LDS stack frames of this kernel
    uint2 spill[rtd::kStack - kK];
    rtd::LdsStackT<kK> S{spill};
    const rtd::GlobalNodes nodes{sc.node};
    const rtd::NodeRec root = rtd::load_node(sc.node, 0);
    // lane state: the runahead kernel keeps TravState, the others share the node / leaf fields
    // (rt_wavefront.h TravStateU)
    std::conditional_t<kSpec, rtd::MegaLane, rtd::MegaLaneU> L;
    L.pix = -1;
    L.state = rtd::M_IDLE;
    // A lane that never gets a pixel still takes part in the shading pass's packing
    // (RT_PACK_TRAV: phase | state << 2 | sp << 5): its phase and stack depth are defined from
    // the start, not the register contents the previous kernel left (a stray phase bit would
    // turn an idle lane's state into TRAV or READY).
    L.T.phase = rtd::TP_POP;
    L.T.sp = 0;
#if defined(RT_DEBUG_CHECKS)
    // debug builds: rt_debug_set_poison(1) leaves out-of-range leftovers in every lane's phase
    // and stack depth instead (the state round 5's fault came from), to show that the packing
    // below masks them and that its check reports them (tests/test_gpu_parity.py)
    if (rt_debug_poison) {
        L.T.phase = 0x7ffffffd;
        L.T.sp = 0x3ffffff;
    }
#endif
    L.wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)threadIdx.x) & ~63u;
    bool exhausted = false;
    bool tail = false, wave_room = false;
#ifdef RT_MEGA_PROF
    unsigned long long pf[7] = {0, 0, 0, 0, 0, 0, 0};
    if (threadIdx.x < 8) rt_prof_lds[threadIdx.x] = 0;
    if (threadIdx.x < 16) rtd::spec_prof_lds[threadIdx.x] = 0;
    if ((threadIdx.x & 63) == 0) rtd::spec_wave_t0_lds[threadIdx.x >> 6] = wall_clock64();
    __syncthreads();
    long long tp = clock64();
    const unsigned long long wt0 = wall_clock64();
    TbAcc tbk;
#endif
    // hand-off resume: the slots past waves * per are taken in the tail (rt_mega.h SpecClaim) by
    // waves below `per` active records
    // (the resume map's address in queue[5], 0 = slot order: read where used)
    rtd::SpecClaim claim{queue + 3, 0, n_items, resume, 0, false, resume ? (const int *)queue[5] : nullptr};
    bool park = false;   // (plain kernel, hand-off: this wave parks its pixels)
    if constexpr (kSpec) {
        if (resume) {
            const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
            const long long dealt = (n_items * resume_pct + 99) / 100;
            const int per = (int)std::min<long long>(64, std::max<long long>(1, (dealt + waves - 1) / waves));
            const long long p = (rtd::mega_slot() >> 6) * per + lane;
            bool xk = false;
            rtd::Rng xs{0u, 0u, 0.f};
            if (lane < per && p < n_items) {
                const rtd::Parked q = rtd::parked_item(resume, claim.ridx, p);
                if (q.pix != rtd::kNoPark) {
                    rtd::mega_resume(L, sc, g, q, root);
                    xk = true;
                    xs = q.x;
                }
            }
            exhausted = true;
            claim.base = waves * per;
            claim.keep = per;
            claim.open = claim.base < n_items;
            if (lane == 0) rtd::spec_hint_take();
            rtd::spec_convert(L, sc, g, rtd::SpecView{(uint4 *)st.mid, st.lanes, rtd::mega_slot() - lane}, lane, xk, xs);
            tail = true;
#ifdef RT_MEGA_PROF
            if (lane == 0) RT_SPEC_STAT(7, 1);
#endif
        }
    }
#if defined(RT_DEBUG_CHECKS)
    unsigned long long dbg_iter = 0;   // debug builds: a wave looping this long reports and leaves
#endif
    for (;;) {
#if defined(RT_DEBUG_CHECKS)
        if (++dbg_iter > (1ull << 22)) {
            const unsigned long long w = (unsigned long long)__popcll(__ballot(L.state == rtd::M_TRAV)) |
                                         (unsigned long long)__popcll(__ballot(L.state == rtd::M_READY)) << 8 |
                                         (unsigned long long)__popcll(__ballot(L.state == rtd::M_DONE)) << 16 |
                                         (unsigned long long)__popcll(__ballot(L.state == rtd::M_DONE_NEW)) << 24 |
                                         (unsigned long long)__popcll(__ballot(L.state == rtd::M_IDLE)) << 32 |
                                         (unsigned long long)tail << 40 | (unsigned long long)park << 41 |
                                         (unsigned long long)exhausted << 42 | (unsigned long long)wave_room << 43;
            RT_CHECK(false, 15, w, (void)0);
            if constexpr (kSpec) {   // the first such wave prints its lanes and records
                const rtd::SpecView V{(uint4 *)st.mid, st.lanes, rtd::mega_slot() - lane};
                const uint4 a = *V.w(0, lane), b = *V.w(1, lane), c = *V.w(2, lane), d = *V.w(3, lane), j = *V.w(4, lane);
                if (atomicAdd(&rt_debug_prints, 1u) < 64u)
                    printf("[stuck] blk %d lane %d state %d pix %d s %d | job tag %u | rec pix %u f %u n %u e %u meta %u tab %08x%08x\n",
                           (int)blockIdx.x, lane, L.state, L.pix, rtd::lane_ctr(L).s, j.x, a.x, a.y, a.z, a.w, b.w, d.w, c.w);
            }
            break;
        }
#endif
        if (!kSpec && !COUNT && !FAST && park) {   // hand-off: lanes idle with a pixel park it
            if (L.state == rtd::M_IDLE && L.pix >= 0) {
                rtd::park_pixel((uint4 *)queue[4], rtd::mega_slot_of(L), L.pix, rtd::lane_ctr(L).s, rtd::lane_rng(L),
                                rtd::lane_sum(L));
                L.pix = -1;
            }
        }
        if (!exhausted) {   // lanes without work take the next items (one atomic per wave)
            const bool need = L.pix < 0 && (kClaimStride == 1 || lane % kClaimStride == 0);
            const unsigned long long m = __ballot(need);
            if (m) {
                const int leader = __ffsll((unsigned long long)m) - 1;
                const unsigned cm = (unsigned)__popcll(m);
                // claiming lanes below this one (mbcnt of the ballot: no per-lane mask held)
                const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                unsigned long long base = 0;
                if (need && below == 0) base = atomicAdd(queue, (unsigned long long)cm);   // the leader
                base = __shfl(base, leader, 64);
                if (need) {
                    const long long p = (long long)base + below;
                    if (p < n_items) {
                        if (FAST) rtd::mega_assign_fast<COUNT>(L, sc, g, p, cs, spp, root, cnt);
                        else rtd::mega_assign<COUNT>(L, sc, g, order ? order[p] : (int)p, root, cnt);
                    }
                }
                if ((long long)base + cm >= n_items) exhausted = true;
            }
        }
        if constexpr (kSpec) {
            if (exhausted && !tail) {
                if (lane == 0) rtd::spec_hint_take();
                rtd::spec_convert(L, sc, g, rtd::SpecView{(uint4 *)st.mid, st.lanes, rtd::mega_slot() - lane}, lane);
                tail = true;
                wave_room = false;
#ifdef RT_MEGA_PROF
                if (lane == 0) RT_SPEC_STAT(7, 1);
#endif
            }
            if (tail) {
                wave_room |= rtd::spec_hint_take();
                if (__any(L.state == rtd::M_DONE_NEW) || (wave_room && __any(L.state == rtd::M_IDLE))) {
#ifdef RT_MEGA_PROF
                    const long long c0 = clock64();
                    tbk.c[5] += 1;
#endif
                    wave_room = rtd::spec_manage(rtd::SpecLanes{L}, sc, g,
                                                 rtd::SpecView{(uint4 *)st.mid, st.lanes, rtd::mega_slot() - lane}, spp,
                                                 out, root, claim);
#ifdef RT_MEGA_PROF
                    if (lane == 0) {
                        RT_SPEC_STAT(0, 1);
                        RT_SPEC_STAT(1, clock64() - c0);
                    }
#endif
                }
                if (!__any(L.state != rtd::M_IDLE)) break;
            } else if (!__any(L.pix >= 0)) {
                break;
            }
        } else if (!__any(L.pix >= 0)) {
            break;
        }
        // hand-off: a wave whose queue is empty and that holds fewer than park_below pixels parks
        // each of them at its next sample end (rt_mega.h mega_shade)
        if (!kSpec && park_below > 0 && exhausted && !park) park = __popcll(__ballot(L.pix >= 0)) < park_below;
        const int nr = __popcll(__ballot(L.state == rtd::M_READY || (LSPLIT && L.state == rtd::M_LREADY)));
        const int nt = __popcll(__ballot(L.state == rtd::M_TRAV || (LSPLIT && L.state == rtd::M_LTRAV)));
        const bool shade_now = nr > 0 && (nr >= (kSpec ? kSpecShadeMin : kShadeMin) || nt == 0);
        // Runahead kernel (the 8-way shards): a traversal iteration issues at priority 1, a
        // shading pass at 0, so waves in their long shading code give issue slots to waves
        // stepping the frame's sample chains: slowest 8-way shard 295 -> 280 ms.  The plain
        // kernel stays at 0 (1 GPU: 1360 -> 1395 ms with the same toggle; 4-way unchanged)
        // (profiles/r02_tail_ab.jsonl).
        if constexpr (kSpec) {
            if (shade_now) __builtin_amdgcn_s_setprio(0);
            else __builtin_amdgcn_s_setprio(1);
        }
#ifdef RT_MEGA_PROF
        {
            const long long t1 = clock64();
            pf[2] += (unsigned long long)(t1 - tp);
            tp = t1;
            pf[shade_now ? 3 : 4] += 1;
            pf[shade_now ? 5 : 6] += (unsigned long long)(shade_now ? nr : nt);
            tbk.at(wt0);
            if (shade_now) {
                tbk.c[3] += 1;
                tbk.c[4] += (unsigned long long)nr;
            }
        }
#endif
        if (!LSPLIT && !shade_now) {
            // Traversal iterations until the wave would shade (the condition above): nothing
            // but trav_step and two ballots per iteration.  In a traversal iteration no lane
            // ends a path, so no lane claims a pixel and a tail wave's runahead records do not
            // change: the outer loop's work between two shading passes is only this.
            int kt = nt;
            int leaf_defer = 0;   // (the runahead kernel's leaf steps deferred in a row: rt_wavefront.h RT_LEAF_DEFER)
            do {
                if (rtd::trav_step_coop<COUNT, kSpec ? kCoopLeavesSpec : kCoopLeavesPlain, kSpec && kSpecMaskLoad,
                                        kSpec ? rtd::kLeafDefer : (COUNT ? 0 : rtd::kLeafDeferPlain)>(
                        sc, L.r, L.T, S, nodes, cnt, L.state == rtd::M_TRAV, kSpec ? st.round_min : kCoopRoundMinPlain,
                        rtd::NoHook{}, &leaf_defer))
                    L.state = rtd::M_READY;
                const unsigned long long rb = __ballot(L.state == rtd::M_READY), tb = __ballot(L.state == rtd::M_TRAV);
                kt = __popcll(tb);
                if (kt == 0 || __popcll(rb) >= (kSpec ? kSpecShadeMin : kShadeMin)) break;
#ifdef RT_MEGA_PROF
                pf[4] += 1;
                pf[6] += (unsigned long long)kt;
                tbk.c[0] += 1;
                tbk.c[1] += (unsigned long long)kt;
                tbk.c[2] += (unsigned long long)__popcll(__ballot(L.state != rtd::M_IDLE));
#endif
            } while (true);
        } else if (kPackTrav && !LSPLIT && !kSpec && !FAST) {
            // shading pass (the inner loop above runs every traversal iteration): a lane that
            // does not shade keeps its phase, stack depth and state packed in one register
            // through the pass (RT_PACK_TRAV).  phase < 4, state < 8 and sp <= kStack hold in
            // every lane (set at the kernel's start, only ever assigned such values; checked in
            // the debug build), and the fields are masked anyway, so that a stray bit of one
            // can never reach another (round 5: an idle lane's leftover phase bit made it READY)
            RT_CHECK((unsigned)L.T.phase < 4u && (unsigned)L.state < 8u && (unsigned)L.T.sp <= (unsigned)rtd::kStack, 14,
                     (unsigned)L.T.phase | (unsigned long long)(unsigned)L.state << 32, (void)0);
            uint32_t pk = ((uint32_t)L.T.phase & 3u) | ((uint32_t)L.state & 7u) << 2 | ((uint32_t)L.T.sp & 127u) << 5;
            asm volatile("" : "+v"(pk));   // (opaque: the compiler cannot fold the unpacking back)
            if (L.state == rtd::M_READY) {
                L.T.phase = 0;   // dead in a READY lane (its stack is empty: T.sp == 0)
                L.T.sp = 0;
                rtd::mega_shade<COUNT, FAST>(L, sc, g, st, spp, out, cost, root, S, cnt, kSpec && tail, park);
            } else {
                L.T.phase = (int)(pk & 3u);
                L.state = (int)((pk >> 2) & 7u);
                L.T.sp = (int)(pk >> 5);
            }
        } else {
            rtd::mega_iterate<COUNT, decltype(S), decltype(nodes), FAST, LSPLIT>(L, shade_now, sc, g, st, spp, out, cost,
                                                                               root, S, nodes, cnt, kSpec && tail);
            // RT_INV_RECOMPUTE: 1 / direction is recomputed after a shading pass (the same IEEE
            // division as make_ray, so the same bits), so a traversing lane does not hold it
            // through the pass's register peak (plain kernel 48 -> 42 spilled VGPRs; 39 with
            // RT_UV_RECOMPUTE; frame -1.5% alone, -2.6% with it: profiles/r05k_ab.jsonl).  0: A/B.
            if (kInvRecompute && shade_now) L.r.inv = rtv::divv(rtd::V3{1.f, 1.f, 1.f}, L.r.d);
        }
        if (kPackTrav && kInvRecompute && !LSPLIT && !kSpec && !FAST && shade_now)
            L.r.inv = rtv::divv(rtd::V3{1.f, 1.f, 1.f}, L.r.d);

#ifdef RT_MEGA_PROF
        {
            const long long t1 = clock64();
            pf[shade_now ? 0 : 1] += (unsigned long long)(t1 - tp);
            tp = t1;
        }
#endif
    }
#ifdef RT_MEGA_PROF
    tbk.flush(tbk.b);
    if (lane == 0) {
        for (int k = 0; k < 7; ++k) atomicAdd(&g_mega_prof[k], pf[k]);
        atomicAdd(&g_mega_prof[7], 1ull);
        const unsigned wi = atomicAdd(&g_wave_n, 1u);
        if (wi < (unsigned)kProfWaves) {
            g_wave_t[2 * wi] = wt0;
            g_wave_t[2 * wi + 1] = wall_clock64();
        }
    }
    __syncthreads();
    if (threadIdx.x < 8) atomicAdd(&g_mega_seg[threadIdx.x], rt_prof_lds[threadIdx.x]);
    if (threadIdx.x < 16) atomicAdd(&rtd::g_spec_prof[threadIdx.x], rtd::spec_prof_lds[threadIdx.x]);
#endif
    rtd::counters_flush<COUNT>(cnt, counters);
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

// Pixel order, step 1: the sort's values (shard pixel ids) and keys (pre-pass costs).
__global__ void __launch_bounds__(256) rt_order_iota_kernel(int *ids, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ids[i] = (int)i;
}

// Pixel order, optional smoothing: box sums of the pre-pass costs over (2r+1) shard pixels
// along a row (dir 0) or down a column (dir 1) of the shard's rows x width grid.
__global__ void __launch_bounds__(256) rt_order_box_kernel(const unsigned *in, unsigned *out, long long n, int width,
                                                           int r, int dir) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const long long rows = n / width, k = p / width, i = p % width;
    unsigned s = 0;
    for (int d = -r; d <= r; ++d) {
        const long long kk = dir ? k + d : k, ii = dir ? i : i + d;
        if (kk >= 0 && kk < rows && ii >= 0 && ii < width) s += in[kk * width + ii];
    }
    out[p] = s;
}

// Pixel order, step 2: `sorted` holds the shard pixels heaviest first.  The first claims of
// the render (each of the `groups` waves takes `per` consecutive queue items at its start, one
// pixel per lane, all lanes at once) get the heaviest m = min(n, groups * per) pixels, spread
// so that every wave holds one pixel of every cost stratum: queue item gi * per + j gets rank
// r = j * a + min(j, b) + gi (m = a * per + b: the ranks in (lane j, wave gi) order of the
// items that exist).  A heavy pixel's wave-mates are then light and finish early, and its
// sequential sample chain runs in a sparse wave.  Later claims stay heaviest-first.
__global__ void __launch_bounds__(256) rt_order_spread_kernel(const int *sorted, int *order, long long n,
                                                              long long groups, long long per) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const long long m = n < groups * per ? n : groups * per;
    long long r = q;
    if (q < m) {
        const long long gi = q / per, j = q % per, a = m / per, b = m % per;
        r = j * a + (j < b ? j : b) + gi;
    }
    order[q] = sorted[r];
}

// Hand-off, between the two launches: the sort keys of the park list's slots, the work a
// parked pixel has left as (samples left) x (its pre-pass estimate + 1); 0 for an empty slot.
// The slots sorted by it, heaviest first, then go through rt_order_spread_kernel, so that the
// runahead launch deals the parked pixels with the most work left one per wave.
__global__ void __launch_bounds__(256) rt_park_keys_kernel(const uint4 *park, long long n, int spp, const unsigned *est,
                                                           unsigned *keys, int *ids) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rtd::Parked q = rtd::parked(park, i);
    unsigned long long k = 0;
    if (q.pix != rtd::kNoPark) k = (unsigned long long)(spp - (int)q.s) * ((unsigned long long)est[q.pix] + 1ull);
    keys[i] = k > 0xffffffffull ? 0xffffffffu : (unsigned)k;
    ids[i] = (int)i;
}
// One 64-bit word, in stream order (the resume map's address in the queue block).
__global__ void rt_set_u64_kernel(unsigned long long *dst, unsigned long long v) { *dst = v; }

// ------------------------------------------------------------------------ wavefront (kernel 4)
// (rt_wavefront.h) init -> { extend ; shade } until every slot has finished its samples.
// Queue modes.  Dense: entry p holds slot p's ray, or an inactive marker (slot -1) once that
// pixel has all its samples; the order never changes, so a wave's lanes keep neighbouring
// pixels (coherent camera rays, coalesced slot-state access) for the whole frame.  Compact:
// active rays only, appended with one atomic per wave; used for the tail of the frame, when
// most slots are finished.  In both modes *count is the number of active rays (the host's
// termination test).
__global__ void __launch_bounds__(256) wf_init_kernel(DevScene sc, ShardGeom g, rtd::WfState st, long long n,
                                                       float4 *qout, unsigned *cout) {
    for (long long base = (long long)blockIdx.x * blockDim.x; base < n; base += (long long)gridDim.x * blockDim.x) {
        const long long i = base + threadIdx.x;
        const bool valid = i < n;
        if (valid) rtd::store_qray(sc, qout, (unsigned)i, (int)i, rtd::wf_init_slot(sc, g, st, i));
        rtd::queue_slot(valid, cout);   // active count
    }
}

// Persistent traversal over the queue: each loop iteration advances every lane of a wave
// by one unit of its own ray's traversal (rt_wavefront.h trav_step).  Lanes whose ray is
// finished idle until kWfRefill of them are idle (or the wave has nothing else to do), then
// take the next rays of the wave's current chunk of the queue; a wave claims a new chunk of
// kWfChunk entries with one atomic when its chunk runs out.  Exit: the claim counter is
// monotonic, so every wave stops claiming once it passes the end and leaves when its lanes
// are done.
template <bool COUNT>
__global__ void __launch_bounds__(256) wf_extend_kernel(DevScene sc, const float4 *qin, const unsigned *count,
                                                         unsigned npos, float4 *hits, unsigned *fetch,
                                                         unsigned *next_count, unsigned long long *counters) {
    const unsigned n = npos ? npos : *count;   // queue positions (dense: all slots)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&counters[7], (unsigned long long)n);  // rays extended
        *next_count = 0;                                 // the shade kernel's output queue
    }
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    uint2 spill[rtd::kStack - rtd::kLdsStackWf];
    rtd::LdsStackT<rtd::kLdsStackWf> S{spill};
    const int lane = threadIdx.x & 63;
    const rtd::GlobalNodes nodes{sc.node};
    const rtd::NodeRec root = rtd::load_node(sc.node, 0);
    unsigned q = 0, lo = 0, hi = 0;   // [lo, hi): the wave's unclaimed part of its chunk
    bool busy = false, exhausted = false;
    rtd::Ray r;
    rtd::TravState T;
    for (;;) {
        const unsigned long long m = __ballot(!busy);
        const unsigned idle = (unsigned)__popcll(m);
        if (!exhausted && (idle >= (unsigned)kWfRefill || idle == 64)) {
            const unsigned rank = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            unsigned got = 0, mine = 0xffffffffu;
            while (got < idle) {
                if (lo >= hi) {
                    unsigned b = 0;
                    if (lane == 0) b = atomicAdd(fetch, kWfChunk);
                    b = __shfl(b, 0, 64);
                    if (b >= n) {
                        exhausted = true;
                        break;
                    }
                    lo = b;
                    hi = b + kWfChunk < n ? b + kWfChunk : n;
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
        if (busy && rtd::trav_step<COUNT>(sc, r, T, S, nodes, cnt)) {
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
                                                        int dense_out, unsigned *fetch, float *out,
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
    const unsigned n = npos ? npos : *cin;   // input positions (dense: all slots)
    if (blockIdx.x == 0 && threadIdx.x == 0) *fetch = 0;   // the next extend launch's claim counter
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
        if (dense_out) {   // (dense out implies dense in: entry q is slot q)
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

// The device image of the scene, built once per scene (every device copies the same bytes).
int ensure_blob(rt_scene *s) {
    if (s->blob) return RT_OK;
    if (s->bvh_depth + 2 >= (uint32_t)rtd::kStack || s->light_bvh_depth + 2 >= (uint32_t)rtd::kStack)
        return rt_fail(RT_ERR_LIMIT, "BVH deeper than the device traversal stack (" + std::to_string(rtd::kStack) + ")");
    if (s->ray_depth > rtd::kMaxDepth) return rt_fail(RT_ERR_LIMIT, "ray_depth exceeds device limit");
    for (size_t k = 0; k < s->node.size() / 8; ++k) {  // traversal frame packing (rt_wavefront.h)
        uint32_t a, b;
        std::memcpy(&a, &s->node[8 * k + 6], 4);
        std::memcpy(&b, &s->node[8 * k + 7], 4);
        if (a >= rtd::kFrameMaxA || b >= 1024u)
            return rt_fail(RT_ERR_LIMIT, "scene too large for the device BVH frame packing (2^22 nodes/triangles, 255 per leaf)");
    }
    auto *b = new rt_device_blob();
    std::vector<uint8_t> &blob = b->bytes;
    // The device copy of the scene BVH is renumbered breadth-first (rt_bvh_layout.h): a
    // node's children stay an adjacent pair (right = left + 1) and leaves keep their triangle
    // ranges, so traversal visits, counters and results are unchanged.  It starts at +32 B so
    // a sibling pair (left odd, left + 1) shares one 64-B line.  Every array starts 256-B
    // aligned: a leaf lane's 4 x 16-B read of the last triangle stays inside the allocation.
    b->o_tri = append(blob, s->tri);
    b->o_attr = append(blob, s->tri_attr);
    b->o_tan = append(blob, s->tri_tan);
    b->o_node = append(blob, rtd::bfs_nodes(s->node), 32);
    b->o_light = append(blob, s->light);
    b->o_lnode = append(blob, s->light_node);
    b->o_mf = append(blob, s->mesh_f);
    b->o_mt = append(blob, s->mesh_tex);
    b->o_nt = append(blob, s->mesh_nt);
    // textures in 4x4-texel tiles (64 B, one cache line): a bilinear 2x2 footprint usually
    // stays in one line instead of always spanning two rows (rt_path.h tex_sample)
    std::vector<uint32_t> tinfo, tiled;
    tile_textures(s->tex_info, s->texels, tinfo, tiled);
    b->o_ti = append(blob, tinfo);
    b->o_tx = append(blob, tiled);
    std::vector<float> lut(512);
    rtd::fill_decode_lut(lut.data());
    b->o_lut = append(blob, lut);
    blob.resize(((blob.size() + 255) & ~size_t(255)) + 256);
    s->blob = b;
    return RT_OK;
}

void free_device_scene(rt_device_scene *d) {
    if (!d) return;
    DeviceGuard guard(d->device);
    if (guard.ok) {
        for (hipStream_t q : {d->fr_stream, d->cp_stream})
            if (q) (void)hipStreamSynchronize(q);
        for (void *p : {d->buf, (void *)d->counters, (void *)d->queue, d->wf_buf, (void *)d->wf_count,
                        (void *)d->wf_fetch, (void *)d->fast_part, d->order_buf, d->fr_buf[0], d->fr_buf[1], d->root_buf})
            if (p) (void)hipFree(p);
        if (d->wf_host_count) (void)hipHostFree(d->wf_host_count);
        for (hipEvent_t e : {d->fr_copied[0], d->fr_copied[1], d->fr_finished, d->fr_last})
            if (e) (void)hipEventDestroy(e);
        for (hipStream_t q : {d->fr_stream, d->cp_stream})
            if (q) (void)hipStreamDestroy(q);
    }
    delete d;
}

// rt_render_frame's per-device streams and events (created once per device copy).
hipError_t ensure_frame_streams(rt_device_scene *d) {
    hipError_t e = hipSuccess;
    if (!d->fr_stream) e = hipStreamCreateWithFlags(&d->fr_stream, hipStreamNonBlocking);
    if (e == hipSuccess && !d->cp_stream) e = hipStreamCreateWithFlags(&d->cp_stream, hipStreamNonBlocking);
    for (hipEvent_t *ev : {&d->fr_copied[0], &d->fr_copied[1], &d->fr_finished, &d->fr_last})
        if (e == hipSuccess && !*ev) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    return e;
}

int ensure_device_scene(rt_scene *s, int device) {
    if (device < 0 || device >= kRtMaxDevices) return rt_fail(RT_ERR_DEVICE, "no HIP device " + std::to_string(device));
    if (s->dev[device]) return RT_OK;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device >= ndev) return rt_fail(RT_ERR_DEVICE, "no HIP device " + std::to_string(device));
    int rc = ensure_blob(s);
    if (rc) return rc;
    const rt_device_blob &b = *s->blob;
    DeviceGuard guard(device);
    if (!guard.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice(" + std::to_string(device) + ") failed");
    rt_device_scene *d = new rt_device_scene();
    d->device = device;
    hipError_t e = hipMalloc(&d->buf, b.bytes.size());
    if (e == hipSuccess) e = hipMemcpy(d->buf, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&d->counters, 16 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void **)&d->queue, 8 * sizeof(unsigned long long));
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        free_device_scene(d);
        return rt_fail(RT_ERR_DEVICE, std::string("scene upload: ") + hipGetErrorString(e));
    }
    d->cu_count = prop.multiProcessorCount;
    uint8_t *base = (uint8_t *)d->buf;
    DevScene &ds = d->ds;
    ds.tri = (const float4 *)(base + b.o_tri);
    ds.tri_attr = (const float4 *)(base + b.o_attr);
    ds.tri_tan = (const float4 *)(base + b.o_tan);
    ds.node = (const float4 *)(base + b.o_node);
    ds.light = (const float4 *)(base + b.o_light);
    ds.light_node = (const float4 *)(base + b.o_lnode);
    ds.mesh_f = (const float *)(base + b.o_mf);
    ds.mesh_tex = (const int *)(base + b.o_mt);
    ds.mesh_nt = (const double *)(base + b.o_nt);
    ds.tex_info = (const uint4 *)(base + b.o_ti);
    ds.texels = (const uint32_t *)(base + b.o_tx);
    ds.lut = (const float *)(base + b.o_lut);
    ds.n_lights = (int)(s->light.size() / 16);
    ds.n_tris = (int)(s->tri.size() / 12);
    ds.n_nodes = (int)(s->node.size() / 8);
    ds.n_meshes = (int)(s->mesh_f.size() / 12);
    ds.ray_depth = s->ray_depth;
    ds.max_distance = s->max_distance;
    ds.width = s->width;
    ds.height = s->height;
    ds.fwidth = (float)s->width;
    ds.fheight = (float)s->height;
    std::memcpy(ds.cam_pos, s->cam_pos, sizeof ds.cam_pos);
    std::memcpy(ds.cam_axes, s->cam_axes, sizeof ds.cam_axes);
    std::memcpy(ds.tan_fov, s->tan_half_fov, sizeof ds.tan_fov);
    s->dev[device] = d;
    return RT_OK;
}

// Workspace: wavefront path state for `n` slots, or the lane-resident kernel's vertex
// records for `n` lane slots, `D` vertices each.
int ensure_wf(rt_device_scene *d, long long n, int D) {
    if (d->wf_buf && d->wf_cap >= n && d->wf_D == D) return RT_OK;
    if (d->wf_buf) (void)hipFree(d->wf_buf);
    d->wf_buf = nullptr;
    d->wf_cap = 0;
    const long long cap = ((n + 255) / 256) * 256;
    const int planes = 8 + 9 * D + 20         // slot state (2 x 16 B), vertex records (36 B each), light-split mid (80 B)
                       + 2 * 4 * rtd::kQRec + 4;   // two ray queues (48 B / entry), hits (16 B / entry)
    const size_t bytes = (size_t)cap * 4 * (size_t)planes;
    HIP_TRY(hipMalloc(&d->wf_buf, bytes));
    if (!d->wf_count) HIP_TRY(hipMalloc((void **)&d->wf_count, 16));
    if (!d->wf_fetch) HIP_TRY(hipMalloc((void **)&d->wf_fetch, 16));
    if (!d->wf_host_count) HIP_TRY(hipHostMalloc((void **)&d->wf_host_count, 16, hipHostMallocDefault));
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
    {   // the hand-off's park list (32 B per lane slot) is the first ray queue (48 B per slot, unused
        // by the lane-resident kernels); its address goes where the kernel reads it (queue[4])
        const unsigned long long park = (unsigned long long)(uintptr_t)d->wf_queue[0];
        HIP_TRY(hipMemcpy(d->queue + 4, &park, sizeof park, hipMemcpyHostToDevice));
    }
    d->wf_cap = cap;
    d->wf_D = D;
    return RT_OK;
}

// 256-thread blocks of `kernel` the device holds at once.
template <class K>
long long resident_blocks(rt_device_scene *d, K kernel) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    return (long long)d->cu_count * per_cu;
}
template <class K>
unsigned persistent_blocks(rt_device_scene *d, K kernel, long long work) {
    const long long need = (work + 255) / 256;
    const long long b = std::min<long long>(need, resident_blocks(d, kernel));
    return (unsigned)std::max<long long>(b, 1);
}

// Per-launch HIP events for RT_FLAG_KERNEL_TIMES (wavefront path).
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

int launch_wavefront(rt_device_scene *d, const ShardGeom &g, int spp, int depth, float *d_out, hipStream_t stream,
                     bool count, LaunchTimer &timer) {
    if (depth < 1 || depth > 15) return rt_fail(RT_ERR_LIMIT, "wavefront path: ray_depth must be in [1, 15]");
    if (spp >= (1 << 20)) return rt_fail(RT_ERR_LIMIT, "wavefront path: spp must be < 2^20");
    if (g.n_pixels >= (1LL << 31)) return rt_fail(RT_ERR_LIMIT, "wavefront path: shards below 2^31 pixels");
    int rc = ensure_wf(d, g.n_pixels, depth);
    if (rc) return rc;
    rtd::WfState w = d->wf;
    w.n = g.n_pixels;
    const long long n = g.n_pixels;
    HIP_TRY(hipMemsetAsync(d->wf_count, 0, 16, stream));
    HIP_TRY(hipMemsetAsync(d->wf_fetch, 0, 16, stream));
    auto extend = count ? wf_extend_kernel<true> : wf_extend_kernel<false>;
    const unsigned ext_blocks = persistent_blocks(d, extend, n);
    const bool mat_lds = d->ds.n_meshes <= kMatLds;
    auto shade = count ? (mat_lds ? wf_shade_kernel<true, true> : wf_shade_kernel<true, false>)
                       : (mat_lds ? wf_shade_kernel<false, true> : wf_shade_kernel<false, false>);
    const unsigned sh_blocks = persistent_blocks(d, shade, n);
    const unsigned init_blocks = (unsigned)std::min<long long>((n + 255) / 256, (long long)d->cu_count * 8);
    hipLaunchKernelGGL(wf_init_kernel, dim3(init_blocks), dim3(256), 0, stream, d->ds, g, w, n, d->wf_queue[0],
                       &d->wf_count[0]);
    HIP_TRY(hipGetLastError());
    bool dense = true, to_compact = false;
    const long long max_iter = (long long)spp * depth + 16;
    int cur = 0;
    for (long long it = 0;; ++it) {
        if (it > max_iter) return rt_fail(RT_ERR_DEVICE, "wavefront path did not drain (internal error)");
        float4 *qi = d->wf_queue[cur], *qo = d->wf_queue[1 - cur];
        const unsigned npos = dense ? (unsigned)n : 0u;
        HIP_TRY(timer.mark(0, stream));
        hipLaunchKernelGGL(extend, dim3(ext_blocks), dim3(256), 0, stream, d->ds, qi, &d->wf_count[cur], npos,
                           d->wf_hits, d->wf_fetch, &d->wf_count[1 - cur], d->counters);
        HIP_TRY(timer.mark(0, stream));
        HIP_TRY(timer.mark(1, stream));
        const int dense_out = dense && !to_compact;
        hipLaunchKernelGGL(shade, dim3(sh_blocks), dim3(256), 0, stream, d->ds, g, w, spp, qi, &d->wf_count[cur], npos,
                           d->wf_hits, qo, &d->wf_count[1 - cur], dense_out, d->wf_fetch, d_out, d->counters);
        if (to_compact) dense = false;
        HIP_TRY(timer.mark(1, stream));
        HIP_TRY(hipGetLastError());
        cur = 1 - cur;
        if ((it & 7) == 7) {   // active rays: done at 0; compact once below kWfCompactBelow
            HIP_TRY(hipMemcpyAsync(d->wf_host_count, &d->wf_count[cur], 4, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (d->wf_host_count[0] == 0) break;
            if (dense && (double)d->wf_host_count[0] < kWfCompactBelow * (double)n) to_compact = true;
        }
    }
    return RT_OK;
}

// Heaviest-first, spread pixel order for a parity-mode render of shard g, built inside the
// frame: a counting fast-mode pre-pass of kOrderSpp samples per pixel measures each pixel's
// traversal work (its own Philox streams: the pre-pass never touches the render's RNG), a
// box filter turns that into an estimate of the pixel's expected work, a radix sort ranks
// the pixels by it, and rt_order_spread_kernel deals the heaviest ones out over the render's
// `groups` waves.  Results never depend on the order; it only shortens the
// frame's tail.  Returns the order in d_order.
int launch_order(rt_device_scene *d, const ShardGeom &g, hipStream_t stream, long long groups, long long per,
                 int **d_order) {
    const long long n = g.n_pixels;
    // order buffer: cost, cost sorted, ids, ids sorted, order (n each), then the sort's scratch
    size_t tmp_bytes = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp_bytes, (unsigned *)nullptr, (unsigned *)nullptr,
                                                         (int *)nullptr, (int *)nullptr, (int)n, 0, 32, stream));
    const size_t arr = (((size_t)n * 4 + 255) / 256) * 256;
    HIP_TRY(grow(&d->order_buf, &d->order_bytes, 5 * arr + tmp_bytes));
    uint8_t *b = (uint8_t *)d->order_buf;
    unsigned *cost = (unsigned *)b, *cost_sorted = (unsigned *)(b + arr);
    int *ids = (int *)(b + 2 * arr), *sorted = (int *)(b + 3 * arr), *order = (int *)(b + 4 * arr);
    void *tmp = b + 5 * arr;
    HIP_TRY(grow((void **)&d->fast_part, &d->fast_part_bytes, (size_t)n * 3 * sizeof(float)));
    HIP_TRY(hipMemsetAsync(d->queue + 1, 0, sizeof(unsigned long long), stream));
    auto pre = rt_mega_kernel<true, true>;
    const unsigned blocks = persistent_blocks(d, pre, n);   // <= ceil(n / 256): lane slots fit the workspace
    rtd::WfState w = d->wf;
    w.n = n;
    w.lanes = (long long)blocks * 256;
    hipLaunchKernelGGL(pre, dim3(blocks), dim3(256), 0, stream, d->ds, g, w, kOrderSpp, d->fast_part,
                       d->counters + 8, d->queue + 1, (const int *)nullptr, cost, kOrderSpp, 0);
    HIP_TRY(hipGetLastError());
    const unsigned nb = (unsigned)((n + 255) / 256);
    if (kOrderRadius > 0) {   // box-filtered costs: the pixel's neighbourhood estimates its expected work
        hipLaunchKernelGGL(rt_order_box_kernel, dim3(nb), dim3(256), 0, stream, (const unsigned *)cost, cost_sorted, n,
                           g.width, kOrderRadius, 0);
        hipLaunchKernelGGL(rt_order_box_kernel, dim3(nb), dim3(256), 0, stream, (const unsigned *)cost_sorted, cost, n,
                           g.width, kOrderRadius, 1);
        HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(rt_order_iota_kernel, dim3(nb), dim3(256), 0, stream, ids, n);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, cost, cost_sorted, ids, sorted, (int)n, 0, 32,
                                                         stream));
    hipLaunchKernelGGL(rt_order_spread_kernel, dim3(nb), dim3(256), 0, stream, (const int *)sorted, order, n, groups,
                       per);
    HIP_TRY(hipGetLastError());
    *d_order = order;
    return RT_OK;
}

// Flag bits outside RT_FLAG_ALL (e.g. ABI 5's RT_FLAG_POOL) are an error, not ignored.
int check_flags(const rt_params *p, const char *who) {
    if (p->flags & ~RT_FLAG_ALL)
        return rt_fail(RT_ERR_ARG, std::string(who) + ": unknown flag bits " + std::to_string(p->flags & ~RT_FLAG_ALL));
    return RT_OK;
}

int launch(rt_scene *s, const rt_params *p, float *d_out, hipStream_t stream, rt_stats *st) {
    if (!s || !p || !d_out) return rt_fail(RT_ERR_ARG, "rt_render: NULL argument");
    if (int rc = check_flags(p, "rt_render")) return rc;
    if (p->device < 0 || p->device >= kRtMaxDevices || !s->dev[p->device])
        return rt_fail(RT_ERR_ARG, "rt_render: scene not uploaded to device " + std::to_string(p->device));
    const int world = p->world > 0 ? p->world : 1, rank = p->rank, rb = p->row_block > 0 ? p->row_block : 8;
    const int spp = p->spp > 0 ? p->spp : s->samples;
    if (spp < 1) return rt_fail(RT_ERR_ARG, "rt_render: samples per pixel must be >= 1");
    if (p->kernel != RT_KERNEL_LANE && p->kernel != RT_KERNEL_WAVEFRONT)
        return rt_fail(RT_ERR_ARG, "rt_render: unknown kernel " + std::to_string(p->kernel) + " (0 lane-resident, 4 wavefront)");
    const bool fast = (p->flags & RT_FLAG_FAST) != 0;
    if ((fast || (p->flags & RT_FLAG_LIGHT_SPLIT)) && p->kernel != RT_KERNEL_LANE)
        return rt_fail(RT_ERR_ARG, "rt_render: fast mode and the light-split kernel run on kernel 0 only");
    if (p->fast_chunk < 0) return rt_fail(RT_ERR_ARG, "rt_render: fast_chunk must be >= 0");
    if ((p->flags & RT_FLAG_NATURAL_ORDER) && (p->flags & RT_FLAG_HEAVY_ORDER))
        return rt_fail(RT_ERR_ARG, "rt_render: RT_FLAG_NATURAL_ORDER and RT_FLAG_HEAVY_ORDER exclude each other");
    if ((int64_t)s->width * s->height > INT32_MAX)
        return rt_fail(RT_ERR_LIMIT, "rt_render: frames above 2^31 pixels are not supported");
    const int64_t rows = rt_shard_rows_impl(s->height, rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    const ShardGeom g = rtd::shard_geom(s->width, rank, world, rb, (long long)rows * s->width);
    rt_device_scene *d = s->dev[p->device];
    DeviceGuard guard(d->device);
    if (!guard.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice failed");
    const bool count = p->count != 0;
    if (count || st) HIP_TRY(hipMemsetAsync(d->counters, 0, 8 * sizeof(unsigned long long), stream));
    LaunchTimer timer;
    timer.on = st != nullptr && (p->flags & RT_FLAG_KERNEL_TIMES) != 0;
    HIP_TRY(hipMemsetAsync(d->queue, 0, sizeof(unsigned long long), stream));
    EventSet events;
    hipEvent_t e0 = nullptr, e_order = nullptr, e1 = nullptr;
    if (st) {
        HIP_TRY(events.make(e0));
        HIP_TRY(events.make(e_order));
        HIP_TRY(events.make(e1));
        HIP_TRY(hipEventRecord(e0, stream));
    }
    bool ordered = false;
    uint64_t sched = 0;   // rt_stats.schedule (RT_SCHED_* bit of the kernel that ran)
    if (g.n_pixels > 0) {
        if (p->kernel == RT_KERNEL_WAVEFRONT) {
            int rc = launch_wavefront(d, g, spp, s->ray_depth, d_out, stream, count, timer);
            if (rc) return rc;
            sched = RT_SCHED_WAVEFRONT;
        } else {   // lane-resident (rt_mega.h), the default
            if (s->ray_depth < 1 || s->ray_depth > 15) return rt_fail(RT_ERR_LIMIT, "ray_depth must be in [1, 15]");
            if (spp >= (1 << 20)) return rt_fail(RT_ERR_LIMIT, "rt_render: spp must be < 2^20");
            // fast mode (RT_FLAG_FAST): work units of `cs` samples, Philox seed per sample, at
            // most kFastMaxChunks units per pixel (partials: pixels x chunks x 12 B)
            int cs = 0, chunks = 1;
            if (fast) {
                cs = std::min(spp, std::max(p->fast_chunk > 0 ? p->fast_chunk : 2, (spp + kFastMaxChunks - 1) / kFastMaxChunks));
                chunks = (spp + cs - 1) / cs;
            }
            const long long n_items = g.n_pixels * chunks;
            const bool lsplit = !fast && (p->flags & RT_FLAG_LIGHT_SPLIT) != 0;
            // Speculative sample runahead (rt_mega.h) where the frame is mostly tail: a shard of
            // at most kSpecPixelsPerLane pixels per resident lane (the 8-way split of the
            // headline: 342 -> 304 ms in round 2; at 4-way, 2 pixels per lane, 359 -> 348 ms in round 3).
            const long long full_blocks = resident_blocks(d, rt_mega_kernel<false, false, false, true>);
            const bool spec = !fast && !lsplit && !count && !(p->flags & RT_FLAG_NO_RUNAHEAD) &&
                              g.n_pixels * kClaimStride <= kSpecPixelsPerLane * full_blocks * 256;
            auto mk = fast ? (count ? rt_mega_kernel<true, true> : rt_mega_kernel<false, true>)
                           : lsplit ? (count ? rt_mega_kernel<true, false, true> : rt_mega_kernel<false, false, true>)
                                    : count ? rt_mega_kernel<true>
                                            : spec ? rt_mega_kernel<false, false, false, true> : rt_mega_kernel<false>;
            sched = fast ? RT_SCHED_FAST : lsplit ? RT_SCHED_LIGHT_SPLIT : spec ? RT_SCHED_RUNAHEAD : RT_SCHED_LANE;
            const bool handoff = !spec && !fast && !lsplit && !count && !(p->flags & RT_FLAG_NO_RUNAHEAD) &&
                                 kClaimStride == 1;
            if (handoff) sched |= RT_SCHED_RUNAHEAD;
            const unsigned blocks = persistent_blocks(d, mk, n_items * kClaimStride);
            const long long slots = (long long)blocks * 256;   // lane slots
            // vertex records are addressed with 32-bit byte offsets (rt_path.h LaneRec)
            if ((unsigned long long)slots * (unsigned long long)s->ray_depth * 32ull >= (1ull << 32))
                return rt_fail(RT_ERR_LIMIT, "rt_render: vertex records beyond 4 GiB");
            int rc = ensure_wf(d, std::max<long long>(g.n_pixels, slots), s->ray_depth);   // vertex records
            if (rc) return rc;
            rtd::WfState w = d->wf;
            w.n = g.n_pixels;
            w.lanes = slots;   // LaneRec slots (<= the workspace capacity)
            if (handoff) {   // the park list: every slot "nothing parked"; the runahead launch's claim counter
                HIP_TRY(hipMemsetAsync(d->wf_queue[0], 0xff, (size_t)slots * 32, stream));
                HIP_TRY(hipMemsetAsync(d->queue + 3, 0, sizeof(unsigned long long), stream));
            }
            w.round_min = d->ds.n_nodes < kCoopRoundNodes ? kCoopRoundMinSpec : 65;
            int *order = nullptr;
            if (!fast && !(p->flags & RT_FLAG_NATURAL_ORDER) && (spp >= kOrderMinSpp || (p->flags & RT_FLAG_HEAVY_ORDER))) {
                // the spread deals one pixel of every cost stratum to each claim of 64 of the
                // launch's first round (one per wave)
                rc = launch_order(d, g, stream, 4LL * blocks, 64, &order);
                if (rc) return rc;
                ordered = true;
            }
            if (st) HIP_TRY(hipEventRecord(e_order, stream));
            float *k_out = d_out;
            if (fast) {
                HIP_TRY(grow((void **)&d->fast_part, &d->fast_part_bytes, (size_t)n_items * 3 * sizeof(float)));
                k_out = d->fast_part;
            }
#ifdef RT_MEGA_PROF
            {
                const unsigned long long z[16] = {};
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mega_prof), z, 8 * sizeof z[0], 0, hipMemcpyHostToDevice, stream));
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mega_seg), z, 8 * sizeof z[0], 0, hipMemcpyHostToDevice, stream));
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(rtd::g_spec_prof), z, sizeof z, 0, hipMemcpyHostToDevice, stream));
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_wave_n), z, sizeof(unsigned), 0, hipMemcpyHostToDevice, stream));
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(rtd::g_chain_n), z, sizeof(unsigned), 0, hipMemcpyHostToDevice, stream));
                static const std::vector<unsigned long long> ztb(kTb * kTbN, 0ull);
                HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tb), ztb.data(), ztb.size() * 8, 0, hipMemcpyHostToDevice, stream));
            }
#endif
            hipLaunchKernelGGL(mk, dim3(blocks), dim3(256), 0, stream, d->ds, g, w, spp, k_out, d->counters, d->queue,
                               (const int *)order, (unsigned *)nullptr, cs, handoff ? kHandoffBelow : 0);
            HIP_TRY(hipGetLastError());
            if (handoff) {   // the parked pixels, on the runahead kernel over the whole resident grid
                // with the pixel order's estimates at hand, the slots heaviest first (work left),
                // spread one per wave (RT_HANDOFF_SPREAD); else slot order
                unsigned long long map = 0;
                if (kHandoffSpread && ordered && slots <= g.n_pixels) {   // (the order buffer holds n_pixels per array)
                    const size_t arr = (((size_t)g.n_pixels * 4 + 255) / 256) * 256;
                    uint8_t *b = (uint8_t *)d->order_buf;
                    const unsigned *est = (const unsigned *)b;   // launch_order's filtered costs
                    unsigned *keys = (unsigned *)(b + arr), *keys_sorted = (unsigned *)(b + 4 * arr);
                    int *ids = (int *)(b + 2 * arr), *ids_sorted = (int *)(b + 3 * arr), *map_p = (int *)(b + arr);
                    void *tmp = b + 5 * arr;
                    size_t tmp_bytes = 0;
                    HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp_bytes, (unsigned *)nullptr,
                                                                         (unsigned *)nullptr, (int *)nullptr, (int *)nullptr,
                                                                         (int)slots, 0, 32, stream));
                    const unsigned nbs = (unsigned)((slots + 255) / 256);
                    hipLaunchKernelGGL(rt_park_keys_kernel, dim3(nbs), dim3(256), 0, stream, (const uint4 *)d->wf_queue[0],
                                       slots, spp, est, keys, ids);
                    HIP_TRY(hipGetLastError());
                    HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, keys, keys_sorted, ids, ids_sorted,
                                                                         (int)slots, 0, 32, stream));
                    // (the runahead launch's static deal: `per` slots to each of its waves, as in the kernel)
                    const long long waves2 = 4LL * full_blocks, dealt = (slots * kHandoffPct + 99) / 100;
                    const long long per2 = std::min<long long>(64, std::max<long long>(1, (dealt + waves2 - 1) / waves2));
                    hipLaunchKernelGGL(rt_order_spread_kernel, dim3(nbs), dim3(256), 0, stream, (const int *)ids_sorted,
                                       map_p, slots, waves2, per2);
                    HIP_TRY(hipGetLastError());
                    map = (unsigned long long)(uintptr_t)map_p;
                }
                hipLaunchKernelGGL(rt_set_u64_kernel, dim3(1), dim3(1), 0, stream, d->queue + 5, map);
                HIP_TRY(hipGetLastError());
                rtd::WfState w2 = w;
                w2.lanes = full_blocks * 256;
                w2.n = slots;   // the park list's slots
                hipLaunchKernelGGL((rt_mega_kernel<false, false, false, true>), dim3((unsigned)full_blocks), dim3(256), 0,
                                   stream, d->ds, g, w2, spp, k_out, d->counters, d->queue, (const int *)nullptr,
                                   (unsigned *)nullptr, 0, kHandoffPct << 8);
                HIP_TRY(hipGetLastError());
            }
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
                             "normal=%.0f mr=%.0f sample=%.0f pdf=%.0f base+brdf=%.0f\n",
                             (double)sg[0] / pf[3], (double)sg[1] / pf[3], (double)sg[2] / pf[3],
                             (double)sg[3] / pf[3], (double)sg[4] / pf[3], (double)sg[5] / pf[3]);
                {   // wave finish times relative to the first wave start: percentiles (ms)
                    unsigned nw = 0;
                    HIP_TRY(hipMemcpyFromSymbolAsync(&nw, HIP_SYMBOL(g_wave_n), sizeof nw, 0, hipMemcpyDeviceToHost, stream));
                    HIP_TRY(hipStreamSynchronize(stream));
                    nw = std::min<unsigned>(nw, (unsigned)kProfWaves);
                    std::vector<unsigned long long> wt(2 * (size_t)nw);
                    if (nw) HIP_TRY(hipMemcpyFromSymbolAsync(wt.data(), HIP_SYMBOL(g_wave_t), wt.size() * 8, 0, hipMemcpyDeviceToHost, stream));
                    HIP_TRY(hipStreamSynchronize(stream));
                    if (nw) {
                        unsigned long long t0 = ~0ull;
                        std::vector<double> ends(nw);
                        for (unsigned i = 0; i < nw; ++i) t0 = std::min(t0, wt[2 * i]);
                        for (unsigned i = 0; i < nw; ++i) ends[i] = (double)(wt[2 * i + 1] - t0) / 1e5;
                        std::sort(ends.begin(), ends.end());
                        std::fprintf(stderr, "[mega prof] wave end ms: p10=%.1f p25=%.1f p50=%.1f p75=%.1f p90=%.1f p99=%.1f max=%.1f\n",
                                     ends[nw / 10], ends[nw / 4], ends[nw / 2], ends[3 * nw / 4], ends[9 * nw / 10],
                                     ends[99 * (size_t)nw / 100], ends[nw - 1]);
                        // per 5-ms bucket: waves alive, traversal iterations per alive wave, lanes per
                        // iteration (traversing, holding work), shading passes, READY lanes per pass,
                        // management passes
                        std::vector<unsigned long long> tbv(kTb * kTbN);
                        HIP_TRY(hipMemcpyFromSymbolAsync(tbv.data(), HIP_SYMBOL(g_tb), tbv.size() * 8, 0, hipMemcpyDeviceToHost, stream));
                        HIP_TRY(hipStreamSynchronize(stream));
                        const int nbk = std::min(kTb, (int)(ends[nw - 1] / 5.0) + 1);
                        for (int b = 0; b < nbk; ++b) {
                            double alive = 0;   // wave-buckets alive (fraction of the bucket)
                            for (unsigned i = 0; i < nw; ++i) {
                                const double s0 = (double)(wt[2 * i] - t0) / 1e5, e0 = (double)(wt[2 * i + 1] - t0) / 1e5;
                                const double lo = std::max(s0, 5.0 * b), hi = std::min(e0, 5.0 * (b + 1));
                                if (hi > lo) alive += (hi - lo) / 5.0;
                            }
                            const unsigned long long *c = &tbv[(size_t)b * kTbN];
                            std::fprintf(stderr, "[mega tb] t=%3d-%3d ms waves=%.0f iters/wave=%.0f trav_lanes=%.1f busy_lanes=%.1f "
                                         "shades/wave=%.1f ready/shade=%.1f passes/wave=%.1f\n", 5 * b, 5 * b + 5, alive,
                                         alive > 0 ? c[0] / alive : 0.0, c[0] ? (double)c[1] / c[0] : 0.0,
                                         c[0] ? (double)c[2] / c[0] : 0.0, alive > 0 ? c[3] / alive : 0.0,
                                         c[3] ? (double)c[4] / c[3] : 0.0, alive > 0 ? c[5] / alive : 0.0);
                        }
                        // the runahead kernel's chain completions: when they end, and where the
                        // last of them stood in the claim order (0 = the first pixel claimed)
                        unsigned nc = 0;
                        HIP_TRY(hipMemcpyFromSymbolAsync(&nc, HIP_SYMBOL(rtd::g_chain_n), sizeof nc, 0, hipMemcpyDeviceToHost, stream));
                        HIP_TRY(hipStreamSynchronize(stream));
                        nc = std::min<unsigned>(nc, (unsigned)rtd::kChainRec);
                        if (nc) {
                            std::vector<unsigned long long> ct(nc);
                            std::vector<unsigned> cpx(nc);
                            HIP_TRY(hipMemcpyFromSymbolAsync(ct.data(), HIP_SYMBOL(rtd::g_chain_t), nc * 8ull, 0, hipMemcpyDeviceToHost, stream));
                            HIP_TRY(hipMemcpyFromSymbolAsync(cpx.data(), HIP_SYMBOL(rtd::g_chain_pix), nc * 4ull, 0, hipMemcpyDeviceToHost, stream));
                            const long long np = g.n_pixels;
                            std::vector<int> rank((size_t)np);
                            if (order) {
                                std::vector<int> ord((size_t)np);
                                HIP_TRY(hipMemcpyAsync(ord.data(), order, (size_t)np * 4, hipMemcpyDeviceToHost, stream));
                                HIP_TRY(hipStreamSynchronize(stream));
                                for (long long q = 0; q < np; ++q)
                                    if (ord[q] >= 0 && ord[q] < np) rank[ord[q]] = (int)q;
                            } else {
                                HIP_TRY(hipStreamSynchronize(stream));
                                for (long long q = 0; q < np; ++q) rank[q] = (int)q;
                            }
                            std::vector<unsigned> ix(nc);
                            for (unsigned q = 0; q < nc; ++q) ix[q] = q;
                            std::sort(ix.begin(), ix.end(), [&](unsigned a, unsigned b) { return ct[a] < ct[b]; });
                            auto ms = [&](unsigned q) { return (double)(ct[ix[q]] - t0) / 1e5; };
                            std::fprintf(stderr, "[mega chains] runahead-kernel chain completions=%u, end ms: p10=%.1f p50=%.1f "
                                         "p90=%.1f p99=%.1f max=%.1f\n", nc, ms(nc / 10), ms(nc / 2), ms(9 * nc / 10),
                                         ms((unsigned)(99ull * nc / 100)), ms(nc - 1));
                            const double fr[4] = {0.5, 0.1, 0.01, 0.001};
                            for (double f : fr) {
                                const unsigned k = std::max(1u, (unsigned)(f * nc));
                                std::vector<double> rr(k);
                                for (unsigned q = 0; q < k; ++q) {
                                    const unsigned px = cpx[ix[nc - 1 - q]];
                                    rr[q] = px < (unsigned)np ? (double)rank[px] / (double)np : -1.0;
                                }
                                std::sort(rr.begin(), rr.end());
                                std::fprintf(stderr, "[mega chains] last %.1f%% (%u chains, from %.1f ms): claim-order position / pixels "
                                             "p10=%.3f p50=%.3f p90=%.3f\n", 100.0 * f, k, ms(nc - k), rr[k / 10], rr[k / 2],
                                             rr[9 * k / 10]);
                            }
                        }
                    }
                }
                unsigned long long sp[16];
                HIP_TRY(hipMemcpyFromSymbolAsync(sp, HIP_SYMBOL(rtd::g_spec_prof), sizeof sp, 0, hipMemcpyDeviceToHost, stream));
                HIP_TRY(hipStreamSynchronize(stream));
                std::fprintf(stderr, "[mega prof] runahead: tail waves=%llu passes/tail wave=%.1f cycles/pass=%.0f "
                             "cycles in passes/wave=%.3g frontier jobs=%llu runahead jobs=%llu added=%llu "
                             "runahead jobs proven=%llu invalidations=%llu\n", sp[7], sp[7] ? (double)sp[0] / sp[7] : 0.0,
                             sp[0] ? (double)sp[1] / sp[0] : 0.0, (double)sp[1] / pf[7], sp[2], sp[3], sp[4], sp[5], sp[6]);
                std::fprintf(stderr, "[mega prof] parked pixels claimed in the tail (hand-off): %llu\n", sp[8]);
                std::fprintf(stderr, "[mega prof] runahead chains: proven share of runahead jobs=%.3f, pixels completed "
                             "in the tail=%llu, mean time per chain link (completion / spp)=%.1f us\n",
                             sp[3] ? (double)sp[5] / (double)sp[3] : 0.0, sp[15], sp[15] ? (double)sp[14] / sp[15] / 100.0 : 0.0);
            }
#endif
        }
        HIP_TRY(hipGetLastError());
    }
    if (st) {
        HIP_TRY(hipEventRecord(e1, stream));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0.f, ms_order = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        if (ordered) HIP_TRY(hipEventElapsedTime(&ms_order, e0, e_order));
        std::memset(st, 0, sizeof *st);
        st->pixels = (uint64_t)g.n_pixels;
        st->samples = (uint64_t)g.n_pixels * (uint64_t)spp;
        st->render_ms = ms;
        st->order_ms = ms_order;
        st->devices = 1;
        st->schedule = sched;
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

// One shard rendered into host memory on the scene's copy on p->device.
int render_host(rt_scene *s, const rt_params *p, float *out, rt_stats *st) {
    int rc = ensure_device_scene(s, p->device);
    if (rc) return rc;
    const int world = p->world > 0 ? p->world : 1, rb = p->row_block > 0 ? p->row_block : 8;
    const int64_t rows = rt_shard_rows_impl(s->height, p->rank, world, rb, nullptr);
    if (rows < 0) return RT_ERR_ARG;
    const size_t bytes = (size_t)rows * s->width * 3 * sizeof(float);
    DeviceGuard guard(p->device);
    if (!guard.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice failed");
    float *d_out = nullptr;
    HIP_TRY(hipMalloc(&d_out, bytes ? bytes : 4));
    rt_stats local;
    rc = launch(s, p, d_out, nullptr, st ? st : &local);
    if (rc == RT_OK) {
        hipError_t e = hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = rt_fail(RT_ERR_DEVICE, std::string("rt_render copy: ") + hipGetErrorString(e));
    }
    (void)hipFree(d_out);
    return rc;
}

}  // namespace

void rt_device_scene_release(rt_scene *s) {
    if (!s) return;
    for (rt_device_scene *&d : s->dev) {
        free_device_scene(d);
        d = nullptr;
    }
    delete s->blob;
    s->blob = nullptr;
}

// Frame assembly on the root device of rt_render_frame (below).
__global__ void __launch_bounds__(256) rt_rows_scatter_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                              const int *__restrict__ frame_row_of, long long rows,
                                                              long long row_bytes) {
    // rows of whole 4-byte words (row_bytes % 4 == 0: W*3 floats, or W*3 bytes with W % 4 == 0)
    // go word by word; other widths byte by byte
    const long long r = blockIdx.y;
    if (r >= rows) return;
    const uint8_t *s = src + r * row_bytes;
    uint8_t *d = dst + (long long)frame_row_of[r] * row_bytes;
    if ((row_bytes & 3) == 0) {
        for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < row_bytes / 4; k += (long long)gridDim.x * blockDim.x)
            ((uint32_t *)d)[k] = ((const uint32_t *)s)[k];
    } else {
        for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < row_bytes; k += (long long)gridDim.x * blockDim.x)
            d[k] = s[k];
    }
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
    // the quantizer thresholds go to each device's constant memory once; threads finishing
    // on the same device at first use serialise on the mutex
    static std::mutex upload_mu;
    static bool uploaded[kRtMaxDevices] = {false};
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= kRtMaxDevices) return rt_fail(RT_ERR_DEVICE, "rt_tonemap_u8_device: device id");
    {
        std::lock_guard<std::mutex> lock(upload_mu);
        if (!uploaded[dev]) {
            HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(k_quant_thr), rtm::kQuantThr, sizeof rtm::kQuantThr));
            uploaded[dev] = true;
        }
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
    if (int rc = check_flags(p, "rt_render")) return rc;
    return render_host(s, p, out, st);
}

// The whole frame as shards 0 .. n-1 of a (world n, row_block) split, shard r on device
// devices[r] (include/rt_hw.h rt_render_frame).  One host thread per distinct device renders
// that device's shards one after another (one render per (scene, device) in flight), finishes
// each to 8 bits on the same device (rt_finish_kernel, scene.cpp:54-64) and copies it, 8-bit
// frame and (if asked) float sums, device-to-device into a staging buffer on the root device
// devices[0] (hipMemcpyPeerAsync: over xGMI between MI355X) on a copy stream of its own, so
// the copy of one shard overlaps the render of the device's next one.  The root then places
// the rows in frame order (rt_rows_scatter_kernel; the reference's canvas, canvas.h:76-89, is
// row-major) behind an event wait per device, and the frame leaves the devices in one copy per
// output.  Streams, events and buffers are kept in the scene's device copies between frames.
// (On the one-GPU pool this runs with every shard on device 0; the peer copies between two
// MI355X have not run on hardware.)
int rt_render_frame(rt_scene *s, const rt_params *p, int32_t n_shards, const int32_t *devices, uint8_t *out_rgb,
                    float *out_sum, rt_stats *st) {
    if (!s || !p || (!out_rgb && !out_sum)) return rt_fail(RT_ERR_ARG, "rt_render_frame: NULL argument");
    if (int rc = check_flags(p, "rt_render_frame")) return rc;
    // (a devices array needs its length: one entry per shard, so n_shards must be given)
    if (devices && n_shards <= 0)
        return rt_fail(RT_ERR_ARG, "rt_render_frame: devices given without n_shards (one device per shard)");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    const int n = n_shards > 0 ? n_shards : ndev;
    if (n < 1 || n > (1 << 16)) return rt_fail(RT_ERR_ARG, "rt_render_frame: bad shard count " + std::to_string(n));
    std::vector<int> dev_of(n);
    for (int r = 0; r < n; ++r) {
        dev_of[r] = devices ? devices[r] : r;
        if (dev_of[r] < 0 || dev_of[r] >= ndev || dev_of[r] >= kRtMaxDevices)
            return rt_fail(RT_ERR_DEVICE, "rt_render_frame: shard " + std::to_string(r) + " on device " +
                                              std::to_string(dev_of[r]) + ", " + std::to_string(ndev) + " visible");
    }
    const int spp = p->spp > 0 ? p->spp : s->samples;
    if (spp < 1) return rt_fail(RT_ERR_ARG, "rt_render_frame: samples per pixel must be >= 1");
    int rc = ensure_blob(s);   // built once here, copied to every device
    if (rc) return rc;
    const int rb = p->row_block > 0 ? p->row_block : 8, W = s->width, H = s->height;
    const int root = dev_of[0];
    // staging on the root: shard r's rows at row offset base[r]; frame_row_of[staging row]
    std::vector<int64_t> rows(n), base(n + 1, 0);
    std::vector<int32_t> frame_row_of((size_t)std::max(H, 1));
    for (int r = 0; r < n; ++r) {
        rows[r] = rt_shard_rows_impl(H, r, n, rb, nullptr);
        if (rows[r] < 0) return rt_fail(RT_ERR_ARG, "rt_render_frame: bad row partition (height " + std::to_string(H) +
                                                        ", row_block " + std::to_string(rb) + ")");
        rt_shard_rows_impl(H, r, n, rb, frame_row_of.data() + base[r]);
        base[r + 1] = base[r] + rows[r];
    }
    const size_t row_u8 = (size_t)W * 3, row_f = row_u8 * sizeof(float);
    std::vector<int> uniq;
    for (int d : dev_of)
        if (std::find(uniq.begin(), uniq.end(), d) == uniq.end()) uniq.push_back(d);
    for (int d : uniq) {   // every device's scene copy, streams and events (kept between frames)
        rc = ensure_device_scene(s, d);
        if (rc) return rc;
        DeviceGuard g(d);
        HIP_TRY(ensure_frame_streams(s->dev[d]));
    }
    // the root's staging (shard r's rows at row offset base[r]), frame buffers and row map:
    // [stage u8 | frame u8 | stage f32 | frame f32 | frame_row_of], each 256-B aligned
    rt_device_scene *rd = s->dev[root];
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t b_u8 = al((size_t)H * row_u8), b_f = out_sum ? al((size_t)H * row_f) : 0,
                 b_map = al((size_t)std::max(H, 1) * sizeof(int32_t));
    {
        DeviceGuard g(root);
        HIP_TRY(grow(&rd->root_buf, &rd->root_bytes, 2 * b_u8 + 2 * b_f + b_map));
        HIP_TRY(hipStreamSynchronize(rd->fr_stream));   // (the previous frame's map upload is done)
        HIP_TRY(hipMemcpyAsync((uint8_t *)rd->root_buf + 2 * b_u8 + 2 * b_f, frame_row_of.data(),
                               (size_t)H * sizeof(int32_t), hipMemcpyHostToDevice, rd->fr_stream));
    }
    uint8_t *stage_u8 = (uint8_t *)rd->root_buf, *frame_u8 = stage_u8 + b_u8;
    uint8_t *stage_f = frame_u8 + b_u8, *frame_f = stage_f + b_f;
    const int *row_map = (const int *)(frame_f + b_f);
    for (int d : uniq) {   // direct xGMI copies between the root and its peers where the runtime allows
        if (d == root) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, d, root) == hipSuccess && can) {
            DeviceGuard g(d);
            (void)hipDeviceEnablePeerAccess(root, 0);
            (void)hipGetLastError();   // (already enabled is not an error here)
        }
        if (hipDeviceCanAccessPeer(&can, root, d) == hipSuccess && can) {
            DeviceGuard g(root);
            (void)hipDeviceEnablePeerAccess(d, 0);
            (void)hipGetLastError();
        }
    }
    std::vector<int> rcs(uniq.size(), RT_OK);
    std::vector<std::string> errs(uniq.size());
    std::vector<rt_stats> sts(n);
    // One host thread per device.  Its shards alternate between two buffers: shard r is
    // rendered (launch waits for it: stats) and finished to 8 bits on the render stream; the
    // copy stream waits for that finish and copies the shard to the root's staging buffer,
    // while the render stream goes on with the next shard in the other buffer (it waits for
    // that buffer's previous copy first).  The device's last copy is marked by fr_last: the
    // root waits for its own on its stream, and for every peer's on the host (below).
    auto work = [&](size_t ui) {
        const int dev = uniq[ui];
        rt_device_scene *dd = s->dev[dev];
        auto fail = [&](int code, const std::string &m) {
            rcs[ui] = rt_fail(code, m);
            errs[ui] = rt_last_error();
        };
        DeviceGuard g(dev);
        if (!g.ok) return fail(RT_ERR_DEVICE, "hipSetDevice failed");
        int64_t max_rows = 0;
        for (int r = 0; r < n; ++r)
            if (dev_of[r] == dev) max_rows = std::max(max_rows, rows[r]);
        const size_t b_sum = al((size_t)max_rows * row_f);
        hipError_t e = hipSuccess;
        for (int b = 0; b < 2 && e == hipSuccess; ++b) e = grow(&dd->fr_buf[b], &dd->fr_bytes[b], b_sum + (size_t)max_rows * row_u8);
        int nb = 0;   // shards done on this device (buffer = nb % 2)
        for (int r = 0; r < n && e == hipSuccess && rcs[ui] == RT_OK; ++r) {
            if (dev_of[r] != dev || rows[r] == 0) continue;
            const int b = nb % 2;
            float *sum = (float *)dd->fr_buf[b];
            uint8_t *rgb = (uint8_t *)dd->fr_buf[b] + b_sum;
            if (nb >= 2) e = hipStreamWaitEvent(dd->fr_stream, dd->fr_copied[b], 0);   // buffer b's last copy done
            if (e != hipSuccess) break;
            rt_params q = *p;
            q.rank = r;
            q.world = n;
            q.row_block = rb;
            q.device = dev;
            q.spp = spp;
            int lr = launch(s, &q, sum, dd->fr_stream, &sts[r]);   // waits (stats)
            if (lr) { rcs[ui] = lr; errs[ui] = rt_last_error(); break; }
            lr = rt_tonemap_u8_device(sum, W, (int32_t)rows[r], spp, rgb, dd->fr_stream);
            if (lr) { rcs[ui] = lr; errs[ui] = rt_last_error(); break; }
            e = hipEventRecord(dd->fr_finished, dd->fr_stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(dd->cp_stream, dd->fr_finished, 0);
            if (e == hipSuccess)
                e = hipMemcpyPeerAsync(stage_u8 + base[r] * row_u8, root, rgb, dev, rows[r] * row_u8, dd->cp_stream);
            if (e == hipSuccess && out_sum)
                e = hipMemcpyPeerAsync(stage_f + base[r] * row_f, root, sum, dev, rows[r] * row_f, dd->cp_stream);
            if (e == hipSuccess) e = hipEventRecord(dd->fr_copied[b], dd->cp_stream);
            ++nb;
        }
        if (e == hipSuccess) e = hipEventRecord(dd->fr_last, dd->cp_stream);
        if (e != hipSuccess && rcs[ui] == RT_OK) fail(RT_ERR_DEVICE, std::string("rt_render_frame: ") + hipGetErrorString(e));
    };
    std::vector<std::thread> threads;
    for (size_t ui = 1; ui < uniq.size(); ++ui) threads.emplace_back(work, ui);
    work(0);
    for (std::thread &t : threads) t.join();
    // every shard's render has ended here (launch waited for each); from now on the host waits
    // only for the copies still in flight, the assembly and the copy to the host: gather_ms
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t ui = 0; ui < uniq.size(); ++ui)
        if (rcs[ui] != RT_OK) {
            for (int d : uniq) {   // (leave no copy in flight into the root's buffers)
                DeviceGuard g(d);
                (void)hipStreamSynchronize(s->dev[d]->cp_stream);
            }
            return rt_fail(rcs[ui], "device " + std::to_string(uniq[ui]) + ": " + errs[ui]);
        }
    {   // assemble on the root behind every device's last copy, one copy to the host per output
        DeviceGuard g(root);
        if (!g.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice failed");
        hipStream_t q = rd->fr_stream;
        // The root's own last copy is waited for on its stream.  A peer's copy is waited for on
        // the host (hipEventSynchronize on the peer's event) before the assembly is queued: a
        // root-stream wait on an event recorded on another device is the cheaper form, but it
        // has not run on a multi-GPU box yet, so the host wait stays the
        // conservative default until it has.
        for (int d : uniq) {
            if (d == root) {
                HIP_TRY(hipStreamWaitEvent(q, s->dev[d]->fr_last, 0));
            } else {
                DeviceGuard gp(d);
                if (!gp.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice failed");
                HIP_TRY(hipEventSynchronize(s->dev[d]->fr_last));
            }
        }
        if (H > 0) {
            hipLaunchKernelGGL(rt_rows_scatter_kernel, dim3(4, (unsigned)H), dim3(256), 0, q, (const uint8_t *)stage_u8,
                               frame_u8, row_map, (long long)H, (long long)row_u8);
            HIP_TRY(hipGetLastError());
            if (out_sum) {
                hipLaunchKernelGGL(rt_rows_scatter_kernel, dim3(8, (unsigned)H), dim3(256), 0, q,
                                   (const uint8_t *)stage_f, frame_f, row_map, (long long)H, (long long)row_f);
                HIP_TRY(hipGetLastError());
            }
        }
        if (out_rgb) HIP_TRY(hipMemcpyAsync(out_rgb, frame_u8, (size_t)H * row_u8, hipMemcpyDeviceToHost, q));
        if (out_sum) HIP_TRY(hipMemcpyAsync(out_sum, frame_f, (size_t)H * row_f, hipMemcpyDeviceToHost, q));
        HIP_TRY(hipStreamSynchronize(q));
    }
    const double gather_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) {
        std::memset(st, 0, sizeof *st);
        std::vector<double> dev_ms(uniq.size(), 0.0), dev_order(uniq.size(), 0.0);   // a device's shards run in turn
        for (int r = 0; r < n; ++r) {
            const rt_stats &x = sts[r];
            st->pixels += x.pixels; st->samples += x.samples; st->rays += x.rays;
            st->aabb_tests += x.aabb_tests; st->tri_tests += x.tri_tests; st->light_queries += x.light_queries;
            st->light_aabb_tests += x.light_aabb_tests; st->light_tri_tests += x.light_tri_tests;
            st->shading_hits += x.shading_hits; st->extend_rays += x.extend_rays;
            st->schedule |= x.schedule;
            const size_t ui = (size_t)(std::find(uniq.begin(), uniq.end(), dev_of[r]) - uniq.begin());
            dev_ms[ui] += x.render_ms;
            dev_order[ui] += x.order_ms;
        }
        st->render_ms = *std::max_element(dev_ms.begin(), dev_ms.end());
        st->order_ms = *std::max_element(dev_order.begin(), dev_order.end());
        st->gather_ms = gather_ms;
        st->devices = (uint64_t)uniq.size();
    }
    return RT_OK;
}

// The float frame over devices 0 .. n-1 (ABI 3 entry; rt_render_frame with shard r on device r).
int rt_render_multi(rt_scene *s, const rt_params *p, int32_t n_devices, float *out, rt_stats *st) {
    if (!s || !p || !out) return rt_fail(RT_ERR_ARG, "rt_render_multi: NULL argument");
    if (int rc = check_flags(p, "rt_render_multi")) return rc;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    const int n = n_devices > 0 ? n_devices : ndev;
    if (n < 1 || n > ndev || n > kRtMaxDevices)
        return rt_fail(RT_ERR_DEVICE, "rt_render_multi: " + std::to_string(n) + " devices requested, " +
                                          std::to_string(ndev) + " visible");
    return rt_render_frame(s, p, n, nullptr, nullptr, out, st);
}

int rt_intersect_rays(rt_scene *s, int64_t n, const float *org, const float *dir, float *out_f, int64_t *out_i) {
    if (!s || n < 0 || (n > 0 && (!org || !dir || !out_f || !out_i))) return rt_fail(RT_ERR_ARG, "rt_intersect_rays: bad argument");
    if (n == 0) return RT_OK;
    int rc = ensure_device_scene(s, 0);
    if (rc) return rc;
    DeviceGuard guard(0);
    if (!guard.ok) return rt_fail(RT_ERR_DEVICE, "hipSetDevice failed");
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
        hipLaunchKernelGGL(rt_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, s->dev[0]->ds,
                           (long long)n, d_o, d_d, d_f, d_i);
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
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(word, HIP_SYMBOL(rt_debug_word), sizeof z));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rt_debug_word), &z, sizeof z));
    return RT_OK;
}
// debug builds only: poison every lane's traversal phase and stack depth at the lane-resident
// kernel's start (rt_mega_kernel), for the packing test
int rt_debug_set_poison(int on) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rt_debug_poison), &on, sizeof on));
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

// rt_device_selfcheck 1: the computed linear texel decode (rt_path.h unorm8) against the IEEE
// division (float)b / 255.f for every byte b, and the packed LDS RNG word (rt_mega.h
// rng_word_pack) round trip over the state range and both normal-cache flags.
__global__ void __launch_bounds__(256) decode_check_kernel(unsigned long long *bad) {
    unsigned long long local = 0;
    if (blockIdx.x == 0) {
        const uint32_t b = threadIdx.x;
        local += __float_as_uint(rtd::unorm8(b)) != __float_as_uint((float)b / 255.f);
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2147483647ull;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i;
#pragma unroll
        for (uint32_t f = 0; f < 2; ++f) {
            uint32_t ux, uf;
            rtd::rng_word_unpack(rtd::rng_word_pack(x, f), ux, uf);
            local += (ux != x) | (uf != f);
        }
    }
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(bad, local);
}

}  // extern "C"

// rt_device_selfcheck 2: the cooperative leaf step (rt_wavefront.h trav_step_coop: four
// helper lanes per leaf lane, DPP quad min with the triangle index as tie-break, NaN t as no
// hit, several leaf rounds) against the per-lane sequential loop of trav_step (the reference's
// in-order strict < of bvh.cpp:226-232 over primitive.cpp:17-57).  Leaves of 1-7 triangles
// over groups rich in exact duplicates (equal t, u, v), coplanar triangles (equal t), NaN and
// infinite vertices; every lane of a 256-thread block is a leaf lane, so each step serves 8 of
// a wave's 64 and the rest wait.  Both round policies (one round per step; rounds until every
// leaf lane is served).  One mismatching field of a case counts once.
template <int kLeaves>
__global__ void __launch_bounds__(256) coop_check_kernel(const float4 *tri, int n_tris, const float4 *nodes,
                                                          const float4 *rays, const uint2 *leaves, int n_cases,
                                                          int round_min, unsigned long long *bad) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const bool valid = i < n_cases;
    DevScene sc{};
    sc.tri = tri;
    sc.n_tris = n_tris;
    sc.node = nodes;
    sc.n_nodes = 2;
    const float4 ro = rays[2 * (valid ? i : 0)], rdv = rays[2 * (valid ? i : 0) + 1];
    const rtd::Ray r = rtd::make_ray(rtv::V3{ro.x, ro.y, ro.z}, rtv::V3{rdv.x, rdv.y, rdv.z});
    const uint2 lf = leaves[valid ? i : 0];
    rtd::TravState T;
    T.best.t = 1e9f;
    T.best.u = T.best.v = 0.f;
    T.best.prim = -1;
    T.acc = 1e9f;
    T.sp = 0;
    T.a = T.b = 0;
    T.k = lf.x;
    T.kend = lf.y;
    T.phase = rtd::TP_LEAF;
    Counters cnt{0, 0, 0, 0, 0, 0, 0};
    uint2 spill[rtd::kStack - 4];
    rtd::LdsStackT<4> S{spill};
    const rtd::GlobalNodes gn{nodes};
    bool active = valid;
    for (int it = 0; it < 64 && __any(active); ++it)   // (bounded: 7 triangles, 64 lanes, 8 per round)
        if (rtd::trav_step_coop<false, kLeaves, false>(sc, r, T, S, gn, cnt, active, round_min)) active = false;
    // the step keeps (t, triangle) only: (u, v) as the shading pass recomputes them
    if (rtd::kUvRecompute && valid && T.best.prim >= 0) rtd::hit_uv(sc, r, T.best);
    // sequential reference: trav_step's per-lane loop, one triangle at a time
    float acc = 1e9f;
    rtd::Hit best{1e9f, 0.f, 0.f, -1};
    for (uint32_t k = lf.x; valid && k < lf.y; ++k) {
        const float4 q0 = tri[3 * k], q1 = tri[3 * k + 1], q2 = tri[3 * k + 2];
        rtd::TriHit h;
        if (rtd::tri_hit_bl(rtv::V3{q0.x, q0.y, q0.z}, rtv::V3{q0.w, q1.x, q1.y}, rtv::V3{q1.z, q1.w, q2.x}, r, h)) {
            acc = h.t < acc ? h.t : acc;
            if (h.t < best.t) best = rtd::Hit{h.t, h.u, h.v, (int)k};
        }
    }
    unsigned long long local = 0;
    if (valid)
        local = (active | (T.best.prim != best.prim) | (__float_as_uint(T.best.t) != __float_as_uint(best.t)) |
                 (__float_as_uint(T.best.u) != __float_as_uint(best.u)) |
                 (__float_as_uint(T.best.v) != __float_as_uint(best.v)) | (__float_as_uint(T.acc) != __float_as_uint(acc)))
                    ? 1ull : 0ull;
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(bad, local);
}

namespace {
// Host-made cases of selfcheck 2 (deterministic): 8-triangle groups of a base triangle, its
// exact copy, a coplanar one behind an equal-t prefix, its copy, a NaN-vertex one, a random
// one, the base again and an infinite-vertex one; rays from random origins at the base's
// centroid (jittered); leaves of 1-7 consecutive triangles.
void coop_cases(std::vector<float> &tri, std::vector<float> &rays, std::vector<uint32_t> &leaves, int n_cases) {
    uint64_t x = 0x9e3779b97f4a7c15ull;
    auto rnd = [&]() {   // [0, 1)
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        return (float)((x >> 40) & 0xffffff) / 16777216.f;
    };
    const int groups = 512;
    tri.assign((size_t)groups * 8 * 12, 0.f);
    std::vector<float> cen((size_t)groups * 3);
    for (int gi = 0; gi < groups; ++gi) {
        float v0[3], U[3], V[3];
        for (int c = 0; c < 3; ++c) {
            v0[c] = rnd() * 4.f - 2.f;
            U[c] = rnd() * 2.f - 1.f;
            V[c] = rnd() * 2.f - 1.f;
            cen[3 * gi + c] = v0[c] + (U[c] + V[c]) / 3.f;
        }
        for (int t = 0; t < 8; ++t) {
            float *o = &tri[((size_t)gi * 8 + t) * 12];
            float a[3], u[3], w[3];
            for (int c = 0; c < 3; ++c) {
                a[c] = v0[c]; u[c] = U[c]; w[c] = V[c];
                if (t == 2 || t == 3) { a[c] = v0[c] + 0.25f * U[c]; }   // same plane, shifted: equal t, other u
                if (t == 5) { a[c] = rnd() * 4.f - 2.f; u[c] = rnd() * 2.f - 1.f; w[c] = rnd() * 2.f - 1.f; }
            }
            if (t == 4) a[1] = __builtin_nanf("");
            if (t == 7) u[0] = __builtin_inff();
            for (int c = 0; c < 3; ++c) { o[c] = a[c]; o[3 + c] = u[c]; o[6 + c] = w[c]; }
        }
    }
    rays.assign((size_t)n_cases * 8, 0.f);
    leaves.assign((size_t)n_cases * 2, 0u);
    for (int i = 0; i < n_cases; ++i) {
        const int gi = (int)(rnd() * groups) % groups;
        float o[3], d[3];
        for (int c = 0; c < 3; ++c) {
            o[c] = rnd() * 20.f - 10.f;
            d[c] = cen[3 * gi + c] + (rnd() - 0.5f) * 0.2f - o[c];
        }
        for (int c = 0; c < 3; ++c) { rays[8 * (size_t)i + c] = o[c]; rays[8 * (size_t)i + 4 + c] = d[c]; }
        const uint32_t len = 1u + (uint32_t)(rnd() * 7.f) % 7u, first = (uint32_t)gi * 8u + (uint32_t)(rnd() * 8.f) % 8u;
        const uint32_t k0 = std::min<uint32_t>(first, (uint32_t)groups * 8u - len);
        leaves[2 * (size_t)i] = k0;
        leaves[2 * (size_t)i + 1] = k0 + len;
    }
}
}  // namespace

extern "C" {

int rt_device_selfcheck(int32_t which, uint64_t *mismatches) {
    if (!mismatches) return rt_fail(RT_ERR_ARG, "rt_device_selfcheck: null output");
    if (which < 0 || which > 2) return rt_fail(RT_ERR_ARG, "rt_device_selfcheck: unknown check " + std::to_string(which));
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, sizeof *d));
    hipError_t e = hipMemset(d, 0, sizeof *d);
    void *cbuf = nullptr;
    if (e == hipSuccess) {
        if (which == 0) {
            hipLaunchKernelGGL(rcp_check_kernel, dim3(4096), dim3(256), 0, nullptr, d);
        } else if (which == 1) {
            hipLaunchKernelGGL(decode_check_kernel, dim3(4096), dim3(256), 0, nullptr, d);
        } else {
            const int n_cases = 1 << 16;
            std::vector<float> tri, rays;
            std::vector<uint32_t> leaves;
            coop_cases(tri, rays, leaves, n_cases);
            const size_t bt = tri.size() * 4 + 64, br = rays.size() * 4, bl = leaves.size() * 4, bn = 256;
            e = hipMalloc(&cbuf, bt + br + bl + bn);
            uint8_t *b = (uint8_t *)cbuf;
            if (e == hipSuccess) e = hipMemset(cbuf, 0, bt + br + bl + bn);
            if (e == hipSuccess) e = hipMemcpy(b, tri.data(), tri.size() * 4, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(b + bt, rays.data(), br, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(b + bt + br, leaves.data(), bl, hipMemcpyHostToDevice);
            const int n_tris = (int)(tri.size() / 12);
            const unsigned blocks = (unsigned)(n_cases / 256);
            if (e == hipSuccess) {
                for (int rm : {65, 1}) {   // one round per step; every leaf lane served in the step
                    hipLaunchKernelGGL(coop_check_kernel<8>, dim3(blocks), dim3(256), 0, nullptr, (const float4 *)b,
                                       n_tris, (const float4 *)(b + bt + br + bl), (const float4 *)(b + bt),
                                       (const uint2 *)(b + bt + br), n_cases, rm, d);
                    hipLaunchKernelGGL(coop_check_kernel<16>, dim3(blocks), dim3(256), 0, nullptr, (const float4 *)b,
                                       n_tris, (const float4 *)(b + bt + br + bl), (const float4 *)(b + bt),
                                       (const uint2 *)(b + bt + br), n_cases, rm, d);
                }
            }
        }
        if (e == hipSuccess) e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (cbuf) (void)hipFree(cbuf);
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

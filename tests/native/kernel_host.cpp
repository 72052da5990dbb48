// kernel_host.cpp — TEST ONLY: compiles the GPU kernel source (raytracing-hw_amd/csrc/rt_path.h)
// for the host so tests can check its arithmetic against the goldens without a GPU.  Not
// part of the product: librt_hw_amd.so has no CPU render path.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include <type_traits>
#include "../../raytracing-hw_amd/csrc/rt_mega.h"
#include "../../raytracing-hw_amd/csrc/rt_bvh_layout.h"
#include "../../include/rt_hw.h"

static rtd::DevScene make(const rt_scene_view *v) {
    rtd::DevScene s{};
    s.tri = (const float4 *)v->tri;
    s.tri_attr = (const float4 *)v->tri_attr;
    s.tri_tan = (const float4 *)v->tri_tan;
    s.node = (const float4 *)v->node;
    // the device copy of the triangles is padded (a leaf lane reads 4 x 16 B of its last
    // triangle: its 3 records and the next one's first)
    static thread_local std::vector<float> tri;
    tri.assign(v->tri, v->tri + 12 * (size_t)v->n_tris);
    tri.resize(tri.size() + 12, 0.f);
    s.tri = (const float4 *)tri.data();
    s.light = (const float4 *)v->light;
    s.light_node = (const float4 *)v->light_node;
    s.mesh_f = v->mesh_f;
    s.mesh_tex = v->mesh_tex;
    s.mesh_nt = v->mesh_normal_transform;
    s.tex_info = (const uint4 *)v->tex_info;
    s.texels = (const uint32_t *)v->texels;
    static float lut[512];
    static bool lut_ready = false;
    if (!lut_ready) { rtd::fill_decode_lut(lut); lut_ready = true; }
    s.lut = lut;
    s.n_lights = (int)v->n_lights;
    s.ray_depth = v->ray_depth;
    s.max_distance = v->max_distance;
    s.width = v->width;
    s.height = v->height;
    s.fwidth = (float)v->width;
    s.fheight = (float)v->height;
    std::memcpy(s.cam_pos, v->cam_pos, sizeof s.cam_pos);
    std::memcpy(s.cam_axes, v->cam_axes, sizeof s.cam_axes);
    std::memcpy(s.tan_fov, v->tan_half_fov, sizeof s.tan_fov);
    return s;
}

// render_pixel (rt_path.h): the reference's recursion order, closest_hit by explicit stack.
extern "C" void kh_render(const rt_scene_view *v, int spp, int64_t p0, int64_t p1, float *out, uint64_t *cnt) {
    rtd::DevScene s = make(v);
    uint64_t c[6] = {0, 0, 0, 0, 0, 0};
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : c[:6])
    for (int64_t p = p0; p < p1; ++p) {
        rtd::Counters k{0, 0, 0, 0, 0, 0, 0};
        rtv::V3 r = rtd::render_pixel<true>(s, (int)(p % v->width), (int)(p / v->width), spp, k);
        out[3 * (p - p0)] = r.x;
        out[3 * (p - p0) + 1] = r.y;
        out[3 * (p - p0) + 2] = r.z;
        c[0] += k.rays; c[1] += k.aabb; c[2] += k.tri; c[3] += k.lq; c[4] += k.laabb; c[5] += k.ltri;
    }
    std::memcpy(cnt, c, sizeof c);
}

// Emulates the wavefront path (wf_init / wf_extend / wf_shade in rt_device.hip) on the host:
// the same rt_wavefront.h slot functions and queue records, driven by a host queue.
extern "C" int kh_render_wf(const rt_scene_view *v, int spp, int rank, int world, int row_block, float *out,
                            uint64_t *cnt_out, int64_t *iterations) {
    rtd::DevScene sc = make(v);
    sc.n_tris = (int)v->n_tris;
    sc.n_nodes = (int)v->n_nodes;
    int64_t rows = 0;
    for (int r = 0; r < v->height; ++r)
        if ((r / row_block) % world == rank) ++rows;
    const long long n = (long long)rows * v->width;
    const rtd::ShardGeom g = rtd::shard_geom(v->width, rank, world, row_block, n);
    const int D = v->ray_depth;
    std::vector<float4> stv((size_t)2 * n), ab((size_t)2 * n * D);
    std::vector<float> cv((size_t)n * D);
    rtd::WfState st{};
    st.n = n;
    st.D = D;
    st.st = stv.data();
    st.rec_ab = ab.data();
    st.rec_c = cv.data();
    std::vector<float4> q((size_t)rtd::kQRec * n), q2((size_t)rtd::kQRec * n), hits((size_t)n);
    unsigned cnt_q = 0;
    for (long long i = 0; i < n; ++i) rtd::store_qray(sc, q.data(), cnt_q++, (int)i, rtd::wf_init_slot(sc, g, st, i));
    rtd::Counters cnt{0, 0, 0, 0, 0, 0, 0};
    uint2 stk[rtd::kStack];
    int64_t it = 0;
    while (cnt_q > 0) {
        if (++it > (int64_t)spp * D + 16) return -1;
        for (unsigned p = 0; p < cnt_q; ++p) {   // extend
            rtd::Hit h;
            rtd::closest_hit_wf<true>(sc, q.data(), p, h, stk, cnt);
            rtd::store_hit(hits.data(), p, h);
        }
        unsigned cnt_q2 = 0;
        for (unsigned p = 0; p < cnt_q; ++p) {   // shade
            int slot;
            rtd::Ray r = rtd::load_qray(q.data(), p, slot);
            const rtd::Hit h = rtd::load_hit(hits.data(), p);
            if (rtd::wf_shade_slot<true>(sc, g, st, spp, slot, r, h, out, cnt)) rtd::store_qray(sc, q2.data(), cnt_q2++, slot, r);
        }
        q.swap(q2);
        cnt_q = cnt_q2;
    }
    uint64_t c[7] = {cnt.rays, cnt.aabb, cnt.tri, cnt.lq, cnt.laabb, cnt.ltri, cnt.hits};
    std::memcpy(cnt_out, c, sizeof c);
    if (iterations) *iterations = it;
    return 0;
}

// SceneDistribution sample + pdf from explicit shading frames (the sampler goldens):
// frame = (point, normal, eye, roughness2); each draw starts from Rng(seed) with an empty
// normal cache; next_out = the engine's next output after the draw (pins draws consumed).
extern "C" void kh_samplers(const rt_scene_view *v, int64_t n, const float *frame, const uint32_t *seed,
                            float *dir_out, float *pdf_out, uint32_t *next_out) {
    rtd::DevScene sc = make(v);
    for (int64_t k = 0; k < n; ++k) {
        const float *f = frame + 10 * k;
        const rtv::V3 pos{f[0], f[1], f[2]}, N{f[3], f[4], f[5]}, eye{f[6], f[7], f[8]};
        rtd::Rng rng{seed[k], 0u, 0.f};
        rtd::Counters cnt{0, 0, 0, 0, 0, 0, 0};
        const rtv::V3 d = rtd::scene_sample(sc, pos, N, eye, f[9], rng);
        pdf_out[k] = rtd::scene_pdf<false>(sc, pos, N, eye, f[9], d, cnt);
        dir_out[3 * k] = d.x;
        dir_out[3 * k + 1] = d.y;
        dir_out[3 * k + 2] = d.z;
        next_out[k] = rtd::rng_next(rng);
    }
}

// Raw sequences: kind 0 = engine outputs, 1 = uniform(-1, 1), 2 = normal(0, 1).
extern "C" void kh_rng(uint32_t seed, int kind, int n, float *out_f, uint32_t *out_u) {
    rtd::Rng rng{seed, 0u, 0.f};
    for (int k = 0; k < n; ++k) {
        if (kind == 0) out_u[k] = rtd::rng_next(rng);
        else if (kind == 1) out_f[k] = rtd::rng_uniform_m11(rng);
        else out_f[k] = rtd::rng_normal(rng);
    }
}

// Emulates rt_mega_kernel (kernel 0): `waves` waves of 64 lanes, round-robin one main-loop
// iteration at a time, sharing the pixel queue, with the kernel's shade_min decision.
// LSPLIT: the light-split kernel (light-pdf walk as lane states M_LTRAV / M_LREADY).
// order (may be NULL): queue item p renders shard pixel order[p], as in the ordered render.
// SPEC: the speculative sample runahead of the waves' tails (rt_mega.h spec_*), driven here
// by host loops over the wave's lanes where the kernel uses ballots (rt_mega.h spec_manage);
// a non-counting render, as on the GPU.
static uint64_t g_spec_passes = 0;   // management passes since the last kh_spec_stats
static int g_static_per_wave = 0;    // > 0: no queue; wave w takes items [w*P, w*P+P) (study of spare lanes)
extern "C" void kh_set_static_per_wave(int p) { g_static_per_wave = p; }
// Hand-off (rt_device.hip RT_HANDOFF): the plain emulation parks (g_park_below > 0) into
// g_park_list by lane slot; the runahead emulation resumes it (g_resume_pct > 0)
static int g_park_below = 0, g_resume_pct = 0;
static std::vector<uint4> g_park_list;
// RT_HANDOFF_SPREAD (rt_device.hip): the resume launch deals the slots heaviest first (work
// left; the harness has no pre-pass estimate, so samples left), spread one per wave
static int g_handoff_spread = 1;
extern "C" void kh_set_handoff_spread(int on) { g_handoff_spread = on; }
static std::vector<int> g_ridx;
// div_magic (rt_wavefront.h) against `/` for divisor d: every n below 2^20, the 2^20 values
// below 2^31, the multiples of d and their neighbours up to 2^31, and `extra` seeded draws;
// returns the number of mismatches.
extern "C" int64_t kh_div_magic_check(uint32_t d, uint32_t extra) {
    uint32_t m = 0;
    int sh = 0;
    rtd::div_magic_make(d, m, sh);
    int64_t bad = 0;
    auto chk = [&](uint64_t n) {
        if (n < (1ull << 31) && (uint64_t)rtd::div_magic((int)n, m, sh) != n / d) ++bad;
    };
    for (uint64_t n = 0; n < (1u << 20); ++n) chk(n);
    for (uint64_t n = (1ull << 31) - (1u << 20); n < (1ull << 31); ++n) chk(n);
    for (uint64_t q = 1; q * d < (1ull << 31) + d && q < (1u << 22); ++q) {
        chk(q * d - 1);
        chk(q * d);
    }
    uint64_t x = 0x9e3779b97f4a7c15ull ^ d;
    for (uint32_t i = 0; i < extra; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        chk(x & 0x7fffffffu);
    }
    return bad;
}

static uint64_t g_rounds = 0;        // main-loop rounds (one iteration of every live wave) of the last render
extern "C" uint64_t kh_rounds() { return g_rounds; }
extern "C" void kh_spec_prof(uint64_t *out) {   // the 16 runahead counters (rt_mega.h RT_SPEC_STAT), not reset
    std::memcpy(out, rtd::g_spec_prof, sizeof rtd::g_spec_prof);
}
extern "C" void kh_spec_stats(uint64_t *out) {   // passes, frontier jobs, runahead jobs, added, invalidations
    out[0] = g_spec_passes;
    out[1] = rtd::g_spec_prof[2];
    out[2] = rtd::g_spec_prof[3];
    out[3] = rtd::g_spec_prof[4];
    out[4] = rtd::g_spec_prof[6];
    g_spec_passes = 0;
    std::memset(rtd::g_spec_prof, 0, sizeof rtd::g_spec_prof);
}

template <bool LSPLIT, bool SPEC = false>
static int render_mega(const rt_scene_view *v, int spp, int rank, int world, int row_block, int waves, int shade_min,
                       const int32_t *order, float *out, uint64_t *cnt_out) {
    rtd::DevScene sc = make(v);
    sc.n_tris = (int)v->n_tris;
    sc.n_nodes = (int)v->n_nodes;
    int64_t rows = 0;
    for (int r = 0; r < v->height; ++r)
        if ((r / row_block) % world == rank) ++rows;
    const long long n = (long long)rows * v->width;
    const rtd::ShardGeom g = rtd::shard_geom(v->width, rank, world, row_block, n);
    const int D = v->ray_depth;
    const long long slots = std::max<long long>(n, (long long)waves * 64);
    std::vector<float4> ab((size_t)2 * slots * D);
    std::vector<float> cv((size_t)slots * D);
    rtd::WfState st{};
    st.n = n;
    st.D = D;
    st.rec_ab = ab.data();
    st.rec_c = cv.data();
    st.lanes = (long long)waves * 64;
    std::vector<float4> mid((size_t)5 * st.lanes);
    st.mid = mid.data();
    const rtd::NodeRec root = rtd::load_node(rtd::mega_nodes(sc), 0);
    const rtd::GlobalNodes nodes{sc.node};
    // lane state as in rt_device.hip: TravState for the runahead kernel, TravStateU otherwise
    using Lane = std::conditional_t<SPEC, rtd::MegaLane, rtd::MegaLaneU>;
    std::vector<Lane> lanes((size_t)waves * 64);
    std::vector<std::vector<uint2>> stacks((size_t)waves * 64, std::vector<uint2>(rtd::kStack));
    for (auto &L : lanes) { L.pix = -1; L.state = rtd::M_IDLE; }
    std::vector<char> exhausted(waves, 0), done(waves, 0), tail(waves, 0), wave_room(waves, 0);
    rtd::Counters cnt{0, 0, 0, 0, 0, 0, 0};
    unsigned long long queue = 0;
    rtd::SpecClaim claim{&queue, 0, 0, nullptr, 0, false};
    // hand-off: parking (plain) / resuming (runahead) as rt_mega_kernel's `mode`
    const bool parking = !SPEC && !LSPLIT && g_park_below > 0, resuming = SPEC && g_resume_pct > 0;
    std::vector<char> park(waves, 0);
    if (parking) g_park_list.assign((size_t)2 * waves * 64, make_uint4(rtd::kNoPark, rtd::kNoPark, rtd::kNoPark, rtd::kNoPark));
    int res_per = 0;
    long long res_n = 0;
    std::vector<char> xk((size_t)waves * 64, 0);
    std::vector<rtd::Rng> xs((size_t)waves * 64);
    if (resuming) {
        res_n = (long long)g_park_list.size() / 2;
        const long long dealt = (res_n * g_resume_pct + 99) / 100;
        res_per = (int)std::min<long long>(64, std::max<long long>(1, (dealt + waves - 1) / waves));
        claim = rtd::SpecClaim{&queue, (long long)waves * res_per, res_n, g_park_list.data(), res_per,
                               (long long)waves * res_per < res_n, nullptr};
        if (g_handoff_spread) {   // rt_park_keys_kernel, the descending sort, rt_order_spread_kernel
            std::vector<std::pair<unsigned, int>> kv((size_t)res_n);
            for (long long i = 0; i < res_n; ++i) {
                const rtd::Parked q = rtd::parked(g_park_list.data(), i);
                kv[(size_t)i] = {q.pix == rtd::kNoPark ? 0u : (unsigned)(spp - (int)q.s), (int)i};
            }
            std::stable_sort(kv.begin(), kv.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
            const long long per = res_per, m = std::min<long long>(res_n, (long long)waves * per), a = m / per, b = m % per;
            g_ridx.resize((size_t)res_n);
            for (long long q = 0; q < res_n; ++q) {
                long long r = q;
                if (q < m) {
                    const long long gi = q / per, j = q % per;
                    r = j * a + (j < b ? j : b) + gi;
                }
                g_ridx[(size_t)q] = kv[(size_t)r].second;
            }
            claim.ridx = g_ridx.data();
        }
    }
    int live = waves;
    g_rounds = 0;
    while (live > 0) {
        ++g_rounds;
        if (g_rounds > 50000000ull) {   // (a schedule that stops draining: report, do not hang the test)
            std::fprintf(stderr, "render_mega: no progress after %llu rounds, %d waves live\n",
                         (unsigned long long)g_rounds, live);
            if constexpr (SPEC) {
                for (int w = 0; w < waves; ++w) {
                    const rtd::SpecView V{(uint4 *)st.mid, st.lanes, (long long)w * 64};
                    for (int l = 0; l < 64; ++l) {
                        const uint4 a = *V.w(0, l), b = *V.w(1, l), c = *V.w(2, l), d = *V.w(3, l);
                        if (b.w & rtd::kRecActive)
                            std::fprintf(stderr, " w%d rec %d: pix %u f %u n %u e %u meta %u tab %08x%08x | lane state %d\n", w, l,
                                         a.x, a.y, a.z, a.w, b.w, d.w, c.w, lanes[(size_t)w * 64 + l].state);
                    }
                }
            }
            return -7;
        }
        for (int w = 0; w < waves; ++w) {
            if (done[w]) continue;
            Lane *W = &lanes[(size_t)w * 64];
            if (parking && park[w])   // lanes idle with a pixel park it (at their lane slot)
                for (int l = 0; l < 64; ++l)
                    if (W[l].state == rtd::M_IDLE && W[l].pix >= 0) {
                        rtd::g_mega_slot = (long long)w * 64 + l;
                        rtd::park_pixel(g_park_list.data(), (long long)w * 64 + l, W[l].pix, rtd::lane_ctr(W[l]).s,
                                        rtd::lane_rng(W[l]), rtd::lane_sum(W[l]));
                        W[l].pix = -1;
                    }
            if (!exhausted[w] && resuming) {   // the park list's slots, res_per per wave
                for (int l = 0; l < res_per; ++l) {
                    const long long p = (long long)w * res_per + l;
                    if (p >= res_n) break;
                    const rtd::Parked q = rtd::parked_item(g_park_list.data(), claim.ridx, p);
                    if (q.pix == rtd::kNoPark) continue;
                    rtd::g_mega_slot = (long long)w * 64 + l;
                    rtd::mega_resume(W[l], sc, g, q, root);
                    xk[(size_t)w * 64 + l] = 1;
                    xs[(size_t)w * 64 + l] = q.x;
                }
                exhausted[w] = 1;
            }
            if (!exhausted[w] && g_static_per_wave > 0) {   // static allotment: wave w renders items [w*P, w*P+P)
                for (int l = 0; l < 64 && l < g_static_per_wave; ++l) {
                    const long long p = (long long)w * g_static_per_wave + l;
                    if (p < n) rtd::mega_assign<!SPEC>(W[l], sc, g, order ? order[p] : (int)p, root, cnt);
                }
                exhausted[w] = 1;
            }
            if (!exhausted[w]) {
                uint64_t m = 0;
                for (int l = 0; l < 64; ++l) if (W[l].pix < 0) m |= 1ull << l;
                if (m) {
                    const long long base = queue;
                    const int cm = __builtin_popcountll(m);
                    queue += cm;
                    for (int l = 0; l < 64; ++l) {
                        if (!(m >> l & 1)) continue;
                        const long long p = base + __builtin_popcountll(m & ((1ull << l) - 1ull));
                        if (p < n) rtd::mega_assign<!SPEC>(W[l], sc, g, order ? order[p] : (int)p, root, cnt);
                    }
                    if (base + cm >= n) exhausted[w] = 1;
                }
            }
            if constexpr (SPEC) {
            if (exhausted[w] && !tail[w]) {
                const rtd::SpecView V{(uint4 *)st.mid, st.lanes, (long long)w * 64};
                rtd::g_mega_slot = (long long)w * 64;
                for (int l = 0; l < 64; ++l) {
                    rtd::g_mega_slot = (long long)w * 64 + l;
                    rtd::spec_convert(W[l], sc, g, V, l, xk[(size_t)w * 64 + l] != 0, xs[(size_t)w * 64 + l]);
                }
                rtd::g_mega_slot = (long long)w * 64;
                rtd::spec_hint_take();
                tail[w] = 1;
                wave_room[w] = 0;
            }
            if (tail[w]) {
                rtd::g_mega_slot = (long long)w * 64;
                wave_room[w] |= rtd::spec_hint_take();
                bool fresh = false, idle = false;
                for (int l = 0; l < 64; ++l) {
                    fresh |= W[l].state == rtd::M_DONE_NEW;
                    idle |= W[l].state == rtd::M_IDLE;
                }
                if (fresh || (wave_room[w] && idle)) {
                    ++g_spec_passes;
                    wave_room[w] = rtd::spec_manage(rtd::SpecLanes{W}, sc, g,
                                                    rtd::SpecView{(uint4 *)st.mid, st.lanes, (long long)w * 64}, spp,
                                                    out, root, claim);
                }
            }
            }
            bool any = false;
            int nr = 0, nt = 0;
            for (int l = 0; l < 64; ++l) {
                any |= tail[w] ? W[l].state != rtd::M_IDLE : W[l].pix >= 0;
                nr += W[l].state == rtd::M_READY || W[l].state == rtd::M_LREADY;
                nt += W[l].state == rtd::M_TRAV || W[l].state == rtd::M_LTRAV;
            }
            if (!any) {
                done[w] = 1;
                --live;
                continue;
            }
            if (parking && exhausted[w] && !park[w]) {
                int held = 0;
                for (int l = 0; l < 64; ++l) held += W[l].pix >= 0;
                park[w] = held < g_park_below;
            }
            const bool shade_now = nr > 0 && (nr >= shade_min || nt == 0);
            for (int l = 0; l < 64; ++l) {
                rtd::ArrayStack S{stacks[(size_t)w * 64 + l].data()};
                rtd::g_mega_slot = (long long)w * 64 + l;
                if (parking)   // (parking renders do not count, as on the GPU)
                    rtd::mega_iterate<false, decltype(S), decltype(nodes), false, LSPLIT>(
                        W[l], shade_now, sc, g, st, spp, out, nullptr, root, S, nodes, cnt, false, (bool)park[w]);
                else
                    rtd::mega_iterate<!SPEC, decltype(S), decltype(nodes), false, LSPLIT>(
                        W[l], shade_now, sc, g, st, spp, out, nullptr, root, S, nodes, cnt, (bool)tail[w]);
            }
        }
    }
    uint64_t c[7] = {cnt.rays, cnt.aabb, cnt.tri, cnt.lq, cnt.laabb, cnt.ltri, cnt.hits};
    std::memcpy(cnt_out, c, sizeof c);
    return 0;
}
extern "C" int kh_render_mega(const rt_scene_view *v, int spp, int rank, int world, int row_block, int waves,
                              int shade_min, const int32_t *order, float *out, uint64_t *cnt_out) {
    return render_mega<false>(v, spp, rank, world, row_block, waves, shade_min, order, out, cnt_out);
}
extern "C" int kh_render_mega_spec(const rt_scene_view *v, int spp, int rank, int world, int row_block, int waves,
                                   int shade_min, const int32_t *order, float *out, uint64_t *cnt_out) {
    return render_mega<false, true>(v, spp, rank, world, row_block, waves, shade_min, order, out, cnt_out);
}
// Hand-off: the plain emulation over `waves` waves parks its sparse tail waves (fewer than
// park_below pixels held once the queue is empty), then the runahead emulation over
// `spec_waves` waves resumes the park list (resume_pct percent dealt at the start).  A
// non-counting render (cnt_out: the counters of the plain part only).
extern "C" int kh_render_mega_handoff(const rt_scene_view *v, int spp, int rank, int world, int row_block, int waves,
                                      int spec_waves, int shade_min, int park_below, int resume_pct,
                                      const int32_t *order, float *out, uint64_t *cnt_out, uint64_t *parked_out) {
    g_park_below = park_below;
    int rc = render_mega<false>(v, spp, rank, world, row_block, waves, shade_min, order, out, cnt_out);
    g_park_below = 0;
    if (rc) return rc;
    uint64_t parked = 0;
    for (size_t k = 0; k < g_park_list.size(); k += 2) parked += g_park_list[k].x != rtd::kNoPark;
    *parked_out = parked;
    g_resume_pct = resume_pct;
    uint64_t c2[7];
    rc = render_mega<false, true>(v, spp, rank, world, row_block, spec_waves, shade_min, nullptr, out, c2);
    g_resume_pct = 0;
    return rc;
}
extern "C" int kh_render_mega_lsplit(const rt_scene_view *v, int spp, int rank, int world, int row_block, int waves,
                                     int shade_min, float *out, uint64_t *cnt_out) {
    return render_mega<true>(v, spp, rank, world, row_block, waves, shade_min, nullptr, out, cnt_out);
}

// rng_skip_sample (rt_path.h, the speculative runahead's state prediction) against the
// real sample chain: for every sample of the listed pixels (parity RNG convention), the state
// the sample ends in must equal rng_skip_sample(start, v) where v is the number of path
// vertices (SceneDistribution::sample calls) of that sample.  stats: [0] samples, [1] states
// that differ, [2] samples with v == ray_depth (the runahead's prediction).
extern "C" void kh_skip_check(const rt_scene_view *v, int spp, int64_t n, const int64_t *pix, uint64_t *stats) {
    rtd::DevScene sc = make(v);
    uint64_t tot = 0, bad = 0, full = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tot, bad, full)
    for (int64_t q = 0; q < n; ++q) {
        const int i = (int)(pix[q] % v->width), j = (int)(pix[q] / v->width);
        const uint32_t seed = (uint32_t)(j * v->width + i) % 2147483647u;
        rtd::Rng rng{seed == 0 ? 1u : seed, 0u, 0.f};
        rtd::Counters cnt{0, 0, 0, 0, 0, 0, 0};
        for (int s = 0; s < spp; ++s) {
            const rtd::Rng start = rng;
            const float ox = rtd::rng_offset(rng), oy = rtd::rng_offset(rng);
            rtd::Ray r = rtd::camera_ray(sc, i, j, ox, oy);
            rtd::PathRec P;
            int nv = 0, power = sc.ray_depth;
            while (power > 0) {   // trace_sample (rt_path.h), keeping the vertex count
                power -= 1;
                rtd::Hit hit;
                const bool ok = rtd::closest_hit<false>(sc, r, hit, cnt);
                if (!(ok && hit.t < sc.max_distance)) break;
                if (!rtd::shade_hit<false>(sc, r, hit, rng, cnt, P, nv)) break;
            }
            rtd::Rng pred = start;
            rtd::rng_skip_sample(pred, nv, sc.n_lights);
            ++tot;
            full += nv == sc.ray_depth;
            uint32_t a, b;
            std::memcpy(&a, &pred.saved, 4);
            std::memcpy(&b, &rng.saved, 4);
            bad += !(pred.x == rng.x && pred.saved_avail == rng.saved_avail && a == b);
        }
    }
    stats[0] = tot;
    stats[1] = bad;
    stats[2] = full;
}

// Per-sample vertex count and traversal cost of the listed pixels (parity RNG convention):
// the data the runahead's prediction of v is measured on (tools/runahead_predict.py).
// nv_out[q*spp + s] = vertices of sample s of pixel q, cost_out[q*spp + s] = its box + triangle tests.
extern "C" void kh_v_trace(const rt_scene_view *v, int spp, int64_t n, const int64_t *pix, uint8_t *nv_out,
                           uint32_t *cost_out) {
    rtd::DevScene sc = make(v);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < n; ++q) {
        const int i = (int)(pix[q] % v->width), j = (int)(pix[q] / v->width);
        const uint32_t seed = (uint32_t)(j * v->width + i) % 2147483647u;
        rtd::Rng rng{seed == 0 ? 1u : seed, 0u, 0.f};
        for (int s = 0; s < spp; ++s) {
            rtd::Counters cnt{0, 0, 0, 0, 0, 0, 0};
            const float ox = rtd::rng_offset(rng), oy = rtd::rng_offset(rng);
            rtd::Ray r = rtd::camera_ray(sc, i, j, ox, oy);
            rtd::PathRec P;
            int nv = 0, power = sc.ray_depth;
            while (power > 0) {
                power -= 1;
                rtd::Hit hit;
                const bool ok = rtd::closest_hit<true>(sc, r, hit, cnt);
                if (!(ok && hit.t < sc.max_distance)) break;
                if (!rtd::shade_hit<true>(sc, r, hit, rng, cnt, P, nv)) break;
            }
            nv_out[q * spp + s] = (uint8_t)nv;
            cost_out[q * spp + s] = (uint32_t)(cnt.aabb + cnt.tri + cnt.laabb + cnt.ltri);
        }
    }
}

// box_pair_hit (rt_wavefront.h) against box_hit_pt on each box of the pair, over `n`
// random cases drawn from a small set of special values (planes through the origin,
// signed zeros, infinities, NaN, inverted boxes) mixed with ordinary floats.  Returns the
// number of mismatching cases (hit flags, far-box inside flag, far-box entry distance bits;
// any NaN distance equals any other: traversal only compares it).
extern "C" long long kh_box_pair_check(long long n, uint32_t seed) {
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    const float specials[] = {0.f, -0.f, 1.f, -1.f, 0.5f, -2.f, 1e-30f, -1e-30f, 1e30f, -1e30f, 1e-45f,
                              __builtin_inff(), -__builtin_inff(), __builtin_nanf("")};
    auto val = [&]() -> float {
        const uint64_t r = next();
        if ((r & 3) == 0) return specials[(r >> 8) % (sizeof specials / sizeof specials[0])];
        return ((float)((r >> 16) & 0xffff) / 32768.f - 1.f) * 4.f;
    };
    long long bad = 0;
    for (long long k = 0; k < n; ++k) {
        rtd::Ray r;
        r.o = rtv::V3{val(), val(), val()};
        r.d = rtv::V3{val(), val(), val()};
        r.inv = rtv::V3{1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z};
        rtd::NodeRec L{}, R{};
        for (int i = 0; i < 3; ++i) {
            const float a = val(), b = val(), c = val(), e = val();
            const bool inv_box = (next() & 15) == 0;   // occasionally inverted
            L.mn[i] = inv_box ? std::max(a, b) : std::min(a, b);
            L.mx[i] = inv_box ? std::min(a, b) : std::max(a, b);
            R.mn[i] = std::min(c, e);
            R.mx[i] = (next() & 7) == 0 ? R.mn[i] : std::max(c, e);   // flat boxes too
            const float oi = i == 0 ? r.o.x : (i == 1 ? r.o.y : r.o.z);
            if ((next() & 7) == 0 && oi <= R.mx[i]) R.mn[i] = oi;   // plane through the origin
        }
        const bool lf = next() & 1;
        float cL[3], cR[3], cF[3];
        bool inL, inR, hL, hR, inF;
        const bool wL = rtd::box_hit_pt(L.mn, L.mx, r, cL, inL);
        const bool wR = rtd::box_hit_pt(R.mn, R.mx, r, cR, inR);
        rtd::box_pair_hit(L, R, r, lf, hL, hR, cF, inF);
        bool ok = wL == hL && wR == hR && inF == (lf ? inR : inL);
        const bool far_hit = lf ? wR : wL;
        if (ok && far_hit) {   // the entry distance is only used for a hit far box
            const float want = rtd::box_dist(lf ? cR : cL, lf ? inR : inL, r), got = rtd::box_dist(cF, inF, r);
            uint32_t a, b;
            std::memcpy(&a, &want, 4);
            std::memcpy(&b, &got, 4);
            ok = ok && (a == b || (want != want && got != got));   // (traversal only compares it)
        }
        bad += !ok;
    }
    return bad;
}

// rt_path.h unorm8 (the device's computed linear texel decode) against (float)b / 255.f for
// every byte, and rt_mega.h's packed LDS RNG word round trip on the state's extremes; returns
// the mismatches.
extern "C" long long kh_decode_check() {
    long long bad = 0;
    for (uint32_t b = 0; b < 256; ++b) {
        const float a = rtd::unorm8(b), want = (float)b / 255.f;
        bad += std::memcmp(&a, &want, 4) != 0;
    }
    const uint32_t xs[] = {0u, 1u, 2u, 48271u, 0x3fffffffu, 0x7ffffffdu, 0x7ffffffeu};
    for (uint32_t x : xs)
        for (uint32_t f = 0; f < 2; ++f) {
            uint32_t ux, uf;
            rtd::rng_word_unpack(rtd::rng_word_pack(x, f), ux, uf);
            bad += (ux != x) | (uf != f);
        }
    return bad;
}

// frt_pool.hpp -- the path megakernel with a per-wave ray pool (included by
// frt_render.hip inside its anonymous namespace: uses DevWork, ItemState,
// lane_rank, scene_to_lds, slot_to_local).
//
// BASELINE north_star: "__ballot/__ffsll wavefront compaction for active-ray
// masks".  In path_megakernel a lane owns one path and traces that path's rays
// one after another (shadow ray, then the extension ray); a lane whose ray is
// done idles in the traversal loop until the wave shades.  Here rays and paths
// are decoupled inside the wave:
//   * a lane OWNS a path (PathState, the item in LDS) and also TRACES one ray
//     (Trav + the ray), which may belong to any path of the wave;
//   * shading queues the path's rays -- the NEE shadow ray S and the extension
//     ray E (path.cpp:45-77, 96-110), both at once -- in two wave-uniform
//     masks (SGPRs): bit j = lane j's path has a ray waiting;
//   * each traversal trip hands the queued rays to the free lanes: ranks by
//     mbcnt over the free-lane ballot, the r-th set bit of the pool mask, the
//     ray's origin / direction pulled from the owner with ds_bpermute;
//   * a finished ray writes its answer to the owner's LDS slot (E: primitive,
//     t, u, v; S: occluded or not); the owner shades once both have landed.
// So S and E of a path trace at the same time in two lanes, and lanes without
// a path of their own (the frame's tail) still trace.  The owner applies the
// shadow answer (L += NEE) before it shades the extension hit, the order
// path_after_shadow keeps, so the film is path_megakernel's bit for bit
// (tests/test_gpu_parity.py::test_ray_pool_matches).
//
// Lambertian / diffuse_light scenes from LDS (the C2 bench plan), fp32.

enum { kRayNone = 0, kRayCam = 1, kRayExt = 2, kRayShadow = 3 };
// item columns: current sample, slot, chunk, pixel, chunk radiance sum (3);
// the item's end sample and the pixel's x, y are derived (min(spp, (chunk+1)
// spi), pixel % nx, pixel / nx), so the pool's per-lane LDS fits 5 blocks/CU
constexpr int kPoolItemWords = 7;
enum { kPiCur, kPiSlot, kPiChunk, kPiPix, kPiAcc };
// answer slots of a lane's path: E primitive + 2 (0 = pending), t, u, v; S 1 =
// unoccluded, 2 = occluded (0 = pending)
constexpr int kPoolSlotWords = 5;
enum { kSlE, kSlT, kSlU, kSlV, kSlS };

// position of the r-th (0-based) set bit of m (r < popcount(m))
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t r)
{
    uint32_t pos = 0, w = (uint32_t)m, c = (uint32_t)__popc(w);
    if (r >= c) { r -= c; pos = 32; w = (uint32_t)(m >> 32); }
#pragma unroll
    for (int s = 16; s >= 1; s >>= 1) {
        c = (uint32_t)__popc(w & ((1u << s) - 1u));
        if (r >= c) { r -= c; pos += s; w >>= s; }
    }
    return pos;
}
// m without its k lowest set bits (wave-uniform)
__device__ __forceinline__ uint64_t drop_lowest(uint64_t m, uint32_t k)
{
    if (k == 0) return m;
    if (k >= (uint32_t)__popcll(m)) return 0;
    const uint32_t p = nth_set_bit(m, k);
    return m & ~((1ull << p) - 1ull);
}
__device__ __forceinline__ float bperm(int src4, float x) { return i2f(__builtin_amdgcn_ds_bpermute(src4, f2i(x))); }

// RESLAB: the slab ray (1/d, -o/d) and t_min again from the traced ray at every
// traversal step instead of kept in Trav (6 VGPRs less across the loop)
template <int STACK, int WORLD, int WAVES, bool RESLAB = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void path_pool_megakernel(
    const DevScene S0, const DevWork W)
{
    // [STACK][kBlock] stack, [kPoolItemWords][kBlock] items, [kPoolSlotWords][kBlock] answer slots, scene
    extern __shared__ __attribute__((aligned(16))) int lds_mem[];
    int *stk = lds_mem + threadIdx.x;
    constexpr int kStackInts = STACK * kBlock, kItemInts = kPoolItemWords * kBlock, kSlotInts = kPoolSlotWords * kBlock;
    DevScene S = S0;
    scene_to_lds<WORLD>(S, lds_mem + kStackInts + kItemInts + kSlotInts);
    const int lane = threadIdx.x & 63;
    int *const slots = lds_mem + kStackInts + kItemInts + (threadIdx.x & ~63);   // + k * kBlock + lane of the wave
    const ItemState I{lds_mem + kStackInts + (int)threadIdx.x};
    const int T2 = W.tile * W.tile;

    // owner role: the lane's path
    PathState<float> P{};       // ro = origin of S and E, rd = E's direction; sd = S's direction
    f3 sd = mk3(0.0f, 0.0f, 0.0f);
    bool have_item = false, exhausted = false, active = false;
    bool waiting = false, e_out = false, s_out = false, has_s = false;
    uint32_t q_cur = 0, q_end = 0;
    // tracer role: the ray this lane traces, for the path of lane t_owner
    Trav<float> T;
    f3 to = mk3(0.0f, 0.0f, 0.0f), td = mk3(0.0f, 0.0f, 1.0f);
    int t_owner = 0, t_kind = kRayNone;
    bool tracing = false;
    int ovf[1];
    uint64_t poolE = 0, poolS = 0;                       // wave-uniform: queued rays by owner lane
    unsigned long long n_cam = 0, n_ext = 0, n_sh = 0, n_smp = 0;

    auto finish_ray = [&]() {                            // the answer to the owner's slot
        if (t_kind == kRayShadow) {
            slots[kSlS * kBlock + t_owner] = T.h.prim < 0 ? 1 : 2;
        } else {
            slots[kSlT * kBlock + t_owner] = f2i(T.h.t);
            slots[kSlU * kBlock + t_owner] = f2i(T.h.u);
            slots[kSlV * kBlock + t_owner] = f2i(T.h.v);
            slots[kSlE * kBlock + t_owner] = T.h.prim + 2;
        }
        t_kind = kRayNone;
    };
    auto queue = [&](bool shadow_too) {                  // this lane's path: E (and S) into the pool
        slots[kSlE * kBlock + lane] = 0;
        slots[kSlS * kBlock + lane] = 0;
        e_out = true;
        s_out = has_s = shadow_too;
        waiting = true;
    };

    for (;;) {
        // ---- traversal: queued rays to free lanes, steps, until the pool is
        // empty and at most trav_min lanes still trace ----
        for (;;) {
            const uint64_t fr = __ballot(!tracing);
            const uint32_t nfree = (uint32_t)__popcll(fr);
            // hand out queued rays once pool_min lanes are free (or the wave is
            // about to shade anyway): the hand-out costs ~60 instructions a trip
            if (fr != 0 && (poolE | poolS) != 0 && (nfree >= (uint32_t)W.pool_min || 64u - nfree <= (uint32_t)W.trav_min)) {
                const uint32_t nS = (uint32_t)__popcll(poolS);
                const uint32_t nE = (uint32_t)__popcll(poolE);
                const uint32_t r = lane_rank(fr);
                const bool take = !tracing && r < nS + nE;
                int owner = lane, kind = kRayNone;
                if (take) {
                    kind = r < nS ? kRayShadow : kRayExt;
                    owner = (int)nth_set_bit(r < nS ? poolS : poolE, r < nS ? r : r - nS);
                }
                // every lane takes part in the pulls (the sources must be active)
                const int src = 4 * owner;
                const f3 o = mk3(bperm(src, P.ro.x), bperm(src, P.ro.y), bperm(src, P.ro.z));
                const f3 de = mk3(bperm(src, P.rd.x), bperm(src, P.rd.y), bperm(src, P.rd.z));
                const f3 ds = mk3(bperm(src, sd.x), bperm(src, sd.y), bperm(src, sd.z));
                const int odepth = __builtin_amdgcn_ds_bpermute(src, P.depth);
                if (take) {
                    to = o;
                    td = kind == kRayShadow ? ds : de;
                    t_owner = owner;
                    t_kind = kind;
                    tracing = trav_begin_world<WORLD>(T, S, to, td, kind == kRayShadow ? 1.0f - kShadowEps : kTMaxClosest);
                    if (!tracing) finish_ray();          // the ray misses the scene box
                }
                const bool cam = take && kind == kRayExt && odepth == 0;
                n_cam += __popcll(__ballot(cam));
                n_ext += __popcll(__ballot(take && kind == kRayExt && !cam));
                n_sh += __popcll(__ballot(take && kind == kRayShadow));
                const uint32_t tS = min(nfree, nS);
                poolS = drop_lowest(poolS, tS);
                poolE = drop_lowest(poolE, min(nfree - tS, nE));
            }
            if constexpr (RESLAB) {
                if (tracing) { T.sr = slab_ray(to, td); T.tmin = bvh_tmin(to); }
            }
            if (tracing && trav_step_world<WORLD, kBlock, STACK>(T, S, to, td, t_kind == kRayShadow, stk, ovf, 0)) {
                tracing = false;
                finish_ray();
            }
            if ((poolE | poolS) == 0 && __popcll(__ballot(tracing)) <= W.trav_min) break;
        }
        // ---- owners: collect the answers; a path whose rays have all landed shades ----
        bool ready = false;
        if (waiting) {
            if (s_out && slots[kSlS * kBlock + lane] != 0) s_out = false;
            if (e_out && slots[kSlE * kBlock + lane] != 0) e_out = false;
            ready = !s_out && !e_out;
        }
        bool next = false;
        if (ready) {
            waiting = false;
            if (has_s && slots[kSlS * kBlock + lane] == 1) P.L = P.L + P.nee;   // path_after_shadow
            const Hit<float> h{slots[kSlE * kBlock + lane] - 2, i2f(slots[kSlT * kBlock + lane]),
                               i2f(slots[kSlU * kBlock + lane]), i2f(slots[kSlV * kBlock + lane])};
            // the sample's RNG key again from the item (not live across the traversal)
            P.key = rng_key(W.seed, (uint32_t)I.get(kPiPix), (uint32_t)(I.get(kPiCur) - 1) + W.s_off);
            uint32_t ne = 0, ns = 0;
            const bool done = path_shade<kMatsNone>(P, S, h, W.max_depth, ne, ns);
            if (done) {
                I.set(kPiAcc + 0, f2i(i2f(I.get(kPiAcc + 0)) + P.L.x));
                I.set(kPiAcc + 1, f2i(i2f(I.get(kPiAcc + 1)) + P.L.y));
                I.set(kPiAcc + 2, f2i(i2f(I.get(kPiAcc + 2)) + P.L.z));
                active = false;
            } else {
                // path_shade set up the shadow ray (P.shadow: ro, rd = S, nxt_d = E's
                // direction from the same origin) or the extension ray alone (ro, rd)
                const bool sh = P.shadow;
                if (sh) {
                    sd = P.rd;
                    P.rd = P.nxt_d;
                    P.shadow = false;
                    ++P.depth;                           // path_after_shadow
                }
                queue(sh);
                next = true;
            }
        }
        // ---- retire a finished item: its chunk sum goes to its own slot ----
        if (!active && have_item && I.get(kPiCur) >= min(W.spp, (I.get(kPiChunk) + 1) * W.spi)) {
            float *dst = W.partial + 3ull * ((size_t)(uint32_t)I.get(kPiChunk) * W.n_slots + (uint32_t)I.get(kPiSlot));
            dst[0] = i2f(I.get(kPiAcc + 0)); dst[1] = i2f(I.get(kPiAcc + 1)); dst[2] = i2f(I.get(kPiAcc + 2));
            have_item = false;
        }
        // ---- wave-aggregated refill (as path_megakernel) ----
        const bool need = !active && !have_item && !exhausted;
        const uint64_t m = __ballot(need);
        if (m) {
            const uint32_t nm = (uint32_t)__popcll(m), rk = lane_rank(m);
            const uint32_t left = q_end - q_cur;
            uint32_t w;
            if (nm <= left) {
                w = q_cur + rk;
                q_cur += nm;
            } else {
                const uint32_t take = max(W.grab, nm - left);
                const int leader = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(W.counter, take);
                base = __shfl(base, leader);
                w = rk < left ? q_cur + rk : base + (rk - left);
                q_cur = base + (nm - left);
                q_end = base + take;
            }
            if (need) {
                if (w >= W.n_items) {
                    exhausted = true;
                } else {
                    const uint32_t s = w % (uint32_t)T2, q = w / (uint32_t)T2;
                    const uint32_t chunk = q % (uint32_t)W.n_chunks, t_ord = q / (uint32_t)W.n_chunks;
                    const int tile_id = W.shard_index + (int)t_ord * W.shard_count;
                    int lx, ly;
                    slot_to_local((int)s, W.tile, lx, ly);
                    const int px = (tile_id % W.ntx) * W.tile + lx, py = (tile_id / W.ntx) * W.tile + ly;
                    if (px < W.nx && py < W.ny) {
                        have_item = true;
                        I.set(kPiCur, (int)chunk * W.spi);
                        I.set(kPiSlot, (int)(t_ord * (uint32_t)T2 + s));
                        I.set(kPiChunk, (int)chunk);
                        I.set(kPiPix, py * W.nx + px);
                        I.set(kPiAcc + 0, 0); I.set(kPiAcc + 1, 0); I.set(kPiAcc + 2, 0);
                    }
                }
            }
        }
        // ---- next camera sample of the item ----
        const bool start = !active && have_item && I.get(kPiCur) < min(W.spp, (I.get(kPiChunk) + 1) * W.spi);
        if (start) {
            const int s_cur = I.get(kPiCur), pix = I.get(kPiPix);
            path_begin(P, S, pix % W.nx, pix / W.nx, W.nx, W.ny, W.seed, (uint32_t)pix, (uint32_t)s_cur + W.s_off);
            I.set(kPiCur, s_cur + 1);
            active = true;
            queue(false);
            next = true;
        }
        n_smp += __popcll(__ballot(start));
        poolS |= __ballot(next && has_s);
        poolE |= __ballot(next);
        if (__ballot(active || !exhausted || tracing) == 0 && (poolE | poolS) == 0) break;
    }
    const unsigned long long c[4] = {n_cam, n_ext, n_sh, n_smp};
    if (lane == 0) {
        const size_t wv = ((size_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
        for (int k = 0; k < 4; ++k) W.wave_rays[4 * wv + k] = c[k];
    }
}

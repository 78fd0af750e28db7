// vr_api.cpp -- host side of libvr.so: module-global device state and the
// C-ABI of include/vr.h (the reference's extern "C" API, K:1889-2406, plus
// the vr_* extensions).  Never exits; errors go to vr_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/vr.h"
#include "vr_internal.h"

namespace {

struct State {
    float *vol = nullptr;
    bool owned = false;
    int nx = 0, ny = 0, nz = 0, nb = 0;
    uint64_t sy = 0, sz = 0;        // record pitch of a voxel row / slice in HBM
    float inv_view[12] = {0};       // __constant__ c_invViewMatrix starts zeroed (K:116)
    hipStream_t stream = nullptr;   // legacy default stream, like the reference
    bool linear_filter = false;     // tex.filterMode = point after initCuda (K:2163)
    std::string err;
    int status = VR_OK;
    // fractal/template codec volume (methods 4/5/6)
    int4 *cb = nullptr;
    float *tpl = nullptr;
    float2 *cerr = nullptr;
    int cnx = 0, cny = 0, cnz = 0, cnb = 0, ntpl = 0, err_slots = 0;
    // flexible blocks (methods 8/9/0): span tables, then the block statistics
    struct Flex {
        int dim = 0, nb = 0, ntpl = 0, nf = 0, ns = 0, nfk = 0, nsk = 0;
        uint64_t *fkeys = nullptr, *skeys = nullptr;
        int32_t *fidx = nullptr, *sidx = nullptr, *scount = nullptr;
        int4 *fcode = nullptr;
        float2 *ferr = nullptr, *shist = nullptr;
        float *tpl = nullptr;
        float4 *blocks = nullptr;
        int nblk = 0;
    } flex;
    // full-frame workgroup -> tile order (frame_order), cached per frame shape
    uint32_t *perm = nullptr;
    size_t perm_cap = 0;
    uint32_t perm_key[22] = {0};
    std::vector<uint32_t> perm_host;
    // adaptive order (frame_order): 0 none, 1 estimate order in use and per-tile
    // costs to be recorded, 2 final; cost_recorded: a render recorded into tile_cost
    int order_state = 0;
    bool cost_recorded = false;
    uint32_t *tile_cost = nullptr;
    size_t tile_cost_cap = 0;
    unsigned long long *wave_clock = nullptr;  // vr_debug_wave_clock (tooling)
    unsigned long long *box_check = nullptr;   // vr_debug_box_check (tooling, -DVR_BOX_CHECK builds)
    // GMM volume (config 5, vr_gmm.hip): planes (w, mu)[voxel][K][2] and
    // sigma[voxel][K] of the resident slices [z_base, z_base + nzs) of an
    // nx x ny x nz volume
    struct Gmm {
        float *wm = nullptr, *sg = nullptr;
        bool owned = false;
        int nx = 0, ny = 0, nz = 0, K = 0, z_base = 0, nzs = 0;
    } gmm;  // the selected slot's volume (vr_gmm_select)
    // the other slot's volume while not selected (a rank of a two-segment slab
    // chain holds a front and a back z-range)
    Gmm gmm_parked[2];
    int gmm_slot = 0;
    // baked statistics (basicDataProcessing / vr_bake_stats, vr_stats.hip):
    // four planes of stats_plane floats for the raw volume (methods 1/2/3 and
    // method 7's corner mean) and
    // of cstats_plane floats for the codec volume (methods 4/5/6); nullptr =
    // not baked, the march decodes the records at every step
    float *stats = nullptr, *cstats = nullptr;
    uint64_t stats_plane = 0, cstats_plane = 0;
    uint64_t stats_sy = 0, stats_sz = 0, cstats_sy = 0, cstats_sz = 0;  // plane_pitches
    // 2x2 (x, y) micro-brick copy of an owned 8-bin volume for the quad march
    // of oblique views (ensure_brick, brick_index); nullptr = not made
    float *brick = nullptr;
    uint64_t bsy = 0, bsz = 0;
    // axis-rows copies of an owned B <= 8 volume for views along y ([0]) and z
    // ([1]) (ensure_axis_copy, axis_copy_strides); nullptr = not made
    struct AxisCopy {
        float *buf = nullptr;
        uint64_t sx = 0, sy = 0, sz = 0, bytes = 0;
    } acopy[2];
    uint64_t brick_bytes = 0;
    // copies of a baked plane (ensure_plane_copy): [axis - 1][plane], axis 1 / 2
    // the y / z-rows copies for views along y or z (k_plane_axis), axis 3 the
    // 8 x 2 x 2 brick copy for oblique views (k_plane8); plane 0-2 = methods 1-3
    struct PlaneCopy {
        float *buf = nullptr;
        uint64_t sy = 0, sz = 0, bytes = 0;
    } pcopy[3][3];
    // layout copies (micro-bricks, axis rows): byte budget (vr_set_layout_budget;
    // UINT64_MAX = the default, layout_budget_bytes) and the cost of the last one
    // made (vr_layout_info)
    uint64_t layout_budget = UINT64_MAX;
    float layout_last_ms = 0.0f;
    uint64_t layout_last_bytes = 0;
    int layout_builds = 0;
    // bumped whenever a resident volume / codec / flexible-block set is
    // released, so an order learned on old data is not reused (the order is a
    // scheduling hint only: any order renders the same image)
    uint32_t volume_epoch = 0;
};

State g;

// Tuning knobs: kernel-path overrides, occupancy caps and layout experiments
// (tests force every kernel path through them; tools sweep them).  Set only
// through vr_set_tuning; the default build never reads the environment, so a
// variable left set in a shell cannot change which kernel runs.  A build with
// -DVR_TUNING also takes unset knobs from the environment (tooling).
std::map<std::string, std::string> g_tuning;

int fail(int status, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g.err = buf;
    g.status = status;
    return status;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(VR_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define VR_HIP(call)                                        \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return hip_fail(e_, #call);   \
    } while (0)

void release_plane_copies();

void release_stats() {
    release_plane_copies();  // copies of the planes go with them
    if (g.stats) (void)hipFree(g.stats);
    g.stats = nullptr;
    g.stats_plane = 0;
}

void release_cstats() {
    if (g.cstats) (void)hipFree(g.cstats);
    g.cstats = nullptr;
    g.cstats_plane = 0;
}

void release_brick() {
    if (g.brick) (void)hipFree(g.brick);
    g.brick = nullptr;
    g.bsy = g.bsz = 0;
    g.brick_bytes = 0;
}

void release_axis_copy(int i) {
    if (g.acopy[i].buf) (void)hipFree(g.acopy[i].buf);
    g.acopy[i] = State::AxisCopy();
}

void release_axis_copy() {
    release_axis_copy(0);
    release_axis_copy(1);
}

void release_plane_copy(int a, int p) {
    if (g.pcopy[a][p].buf) (void)hipFree(g.pcopy[a][p].buf);
    g.pcopy[a][p] = State::PlaneCopy();
}

void release_plane_copies() {
    for (int a = 0; a < 3; a++)
        for (int p = 0; p < 3; p++) release_plane_copy(a, p);
}

uint64_t layout_resident() {
    uint64_t b = g.brick_bytes + g.acopy[0].bytes + g.acopy[1].bytes;
    for (int a = 0; a < 3; a++)
        for (int p = 0; p < 3; p++) b += g.pcopy[a][p].bytes;
    return b;
}

// Room for a layout copy of `bytes`: within the budget (vr_set_layout_budget)
// next to the copies already resident (less `freed`, a copy the caller would
// drop first), and HBM keeps max(4 GiB, 5 %) free after it for the caller.
// The default budget: two copies of the resident record volume (a brick copy
// and one axis copy, or both axis copies) plus three copies of one baked plane,
// each with 1/8 for the copies' padding -- what one view class plus one change
// of view needs, not every copy at once (a third record copy replaces one).
// Plus 64 MiB: a volume a few cells wide pads its 2 x 2 micro-bricks by up to
// 4x, far beyond 1/8, and copies that small cost nothing worth refusing.
uint64_t layout_budget_bytes() {
    if (g.layout_budget != UINT64_MAX) return g.layout_budget;
    const uint64_t rec = g.vol ? g.sz * (uint64_t)g.nz * g.nb * sizeof(float) : 0;
    const uint64_t plane = g.stats ? g.stats_plane * sizeof(float) : 0;
    return 2 * (rec + rec / 8) + 3 * (plane + plane / 8) + (64ull << 20);
}

bool layout_room(uint64_t bytes, uint64_t freed = 0) {
    const uint64_t have = layout_resident() - freed;
    const uint64_t budget = layout_budget_bytes();
    if (budget < have || budget - have < bytes) return false;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return (uint64_t)free_b + freed >= bytes + std::max<uint64_t>(4ull << 30, total_b / 20);
}

void release_volume() {
    release_stats();
    release_brick();
    release_axis_copy();
    g.volume_epoch++;
    if (g.vol && g.owned) (void)hipFree(g.vol);
    g.vol = nullptr;
    g.owned = false;
    g.nx = g.ny = g.nz = g.nb = 0;
    g.sy = g.sz = 0;
}

// Row / slice pitch (in records) of the resident volume.  VR_PAD="px,pz" adds
// px records to every row and pz records to every slice (layout experiments).
void choose_pitch(int nx, int ny, uint64_t &sy, uint64_t &sz) {
    long px = 0, pz = 0;
    if (const char *e = vr::tuning("VR_PAD")) {
        char *end = nullptr;
        px = std::strtol(e, &end, 10);
        if (end && *end == ',') pz = std::strtol(end + 1, nullptr, 10);
        if (px < 0 || px > 4096) px = 0;
        if (pz < 0 || pz > (1 << 20)) pz = 0;
    }
    sy = (uint64_t)nx + (uint64_t)px;
    sz = sy * (uint64_t)ny + (uint64_t)pz;
}

float entropy_norm(int nb) {
    // K:769: log((float)nBins) / log(2.0f) with the float overloads of log
    const float a = (float)std::log((double)(float)nb);
    const float b = (float)std::log((double)2.0f);
    return a / b;
}

uint32_t tiles_x(uint32_t w) { return (w + vr::kTileW - 1) / vr::kTileW; }
uint32_t tiles_y(uint32_t h) { return (h + vr::kTileH - 1) / vr::kTileH; }

void release_codec() {
    release_cstats();
    g.volume_epoch++;
    if (g.cb) (void)hipFree(g.cb);
    if (g.tpl) (void)hipFree(g.tpl);
    if (g.cerr) (void)hipFree(g.cerr);
    g.cb = nullptr;
    g.tpl = nullptr;
    g.cerr = nullptr;
    g.cnx = g.cny = g.cnz = g.cnb = g.ntpl = g.err_slots = 0;
}

void release_flex_blocks() {
    g.volume_epoch++;
    if (g.flex.blocks) (void)hipFree(g.flex.blocks);
    g.flex.blocks = nullptr;
    g.flex.nblk = 0;
}

void release_flex() {
    release_flex_blocks();
    void *ptrs[] = {g.flex.fkeys, g.flex.skeys, g.flex.fidx, g.flex.sidx, g.flex.scount,
                    g.flex.fcode, g.flex.ferr, g.flex.shist, g.flex.tpl};
    for (void *q : ptrs)
        if (q) (void)hipFree(q);
    g.flex = State::Flex();
}

bool is_flex_method(int m) { return m == 8 || m == 9 || m == 0; }

int check_method(int m) {
    if (m == 1 || m == 2 || m == 3 || m == 7 || m == 4 || m == 5 || m == 6) return VR_OK;
    if (is_flex_method(m)) {
        if (!g.flex.blocks)
            return fail(VR_ERR_STATE,
                        "queryMethod %d needs the flexible-block statistics (span tables via "
                        "initCuda / vr_init_flex, then dataProcessing / vr_flex_process)", m);
        return VR_OK;
    }
    return fail(VR_ERR_ARG, "unknown queryMethod %d", m);
}

// Host estimate of the samples a ray takes before leaving the volume (the
// slab test of K:136-156 on the pixel's ray; early termination ignored).
float est_steps(const float *M, uint32_t W, uint32_t H, float x, float y) {
    const float u = (x / (float)W) * 2.0f - 1.0f, v = (y / (float)H) * 2.0f - 1.0f;
    const float inv = 1.0f / std::sqrt(u * u + v * v + 4.0f);
    const float ax = u * inv, ay = v * inv, az = -2.0f * inv;
    const float d[3] = {ax * M[0] + ay * M[1] + az * M[2], ax * M[4] + ay * M[5] + az * M[6],
                        ax * M[8] + ay * M[9] + az * M[10]};
    const float o[3] = {M[3], M[7], M[11]};
    float tn = -1e30f, tf = 1e30f;
    for (int k = 0; k < 3; k++) {
        const float a = (-1.0f - o[k]) / d[k], b = (1.0f - o[k]) / d[k];
        tn = std::max(tn, std::min(a, b));
        tf = std::min(tf, std::max(a, b));
    }
    tn = std::max(tn, 0.0f);
    return tf > tn ? (tf - tn) / vr::kTStep : 0.0f;
}

// Full-frame tile order.  Workgroup b runs on XCD b % 8, and each XCD has its
// own L2.  Tiles are grouped in bx x by blocks (neighbouring tiles share the
// records along their common edges, so a block keeps that sharing inside one
// L2); block (i, j) goes to XCD (i + 3 j) % 8, a diagonal lattice that gives
// every XCD an evenly spread eighth of any region spanning a few blocks -- so
// the hit region, and with it the ray-marching work, is split evenly (a raster
// split hands the frame's empty top and bottom strips to whole XCDs).  Each
// XCD takes its blocks longest-ray first (longest-processing-time order on
// the view's ray lengths): a tile's march is a chain of dependent gathers, so
// the frame ends no earlier than its longest tile started plus that tile's
// length.  VR_XBLOCK="bx,by" (default 1,4 = 64x16 pixels; "0" = plain raster
// order).
//
// Adaptive refinement: the estimate ignores early ray termination and the
// volume's content, so the first render of a view also records every tile's
// measured cost (per wave: its longest ray's samples + 2, record_tile_cost),
// and the next render of the same view re-deals the blocks by those costs
// (lists_from_costs).  VR_NO_ADAPT keeps the estimate order.

// Interleave the 8 per-XCD lists into the workgroup order (entry b runs on
// XCD b % 8) and upload it as g.perm.
int upload_perm(const std::vector<std::vector<uint32_t>> &lists) {
    std::vector<uint32_t> &h = g.perm_host;
    h.clear();
    size_t longest = 0;
    for (auto &l : lists) longest = std::max(longest, l.size());
    for (size_t i = 0; i < longest; i++)
        for (auto &l : lists)
            if (i < l.size()) h.push_back(l[i]);
    if (h.size() > g.perm_cap) {  // grow; otherwise rewrite in stream order
        if (g.perm) (void)hipFree(g.perm);
        g.perm = nullptr;
        g.perm_cap = 0;
        VR_HIP(hipMalloc(&g.perm, h.size() * sizeof(uint32_t)));
        g.perm_cap = h.size();
    }
    VR_HIP(hipMemcpyAsync(g.perm, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          g.stream));
    return VR_OK;
}

// Measured-cost deal: blocks sorted by total cost, each given to the least
// loaded XCD that still has room (every XCD keeps the same number of blocks,
// +-1, so the interleaved order keeps entry b on XCD b % 8); an XCD's blocks
// stay in dealing order, i.e. most expensive first.
void lists_from_costs(const std::vector<uint32_t> &cost, uint32_t tx, uint32_t ty, uint32_t bx,
                      uint32_t by, std::vector<std::vector<uint32_t>> &lists) {
    const uint32_t nbx = (tx + bx - 1) / bx, nby = (ty + by - 1) / by;
    struct Blk { uint64_t cost; uint32_t i, j; };
    std::vector<Blk> blk;
    blk.reserve((size_t)nbx * nby);
    for (uint32_t j = 0; j < nby; j++)
        for (uint32_t i = 0; i < nbx; i++) {
            uint64_t c = 0;
            for (uint32_t y = j * by; y < std::min(ty, j * by + by); y++)
                for (uint32_t x = i * bx; x < std::min(tx, i * bx + bx); x++)
                    c += cost[(size_t)y * tx + x];
            blk.push_back({c, i, j});
        }
    std::stable_sort(blk.begin(), blk.end(), [](const Blk &a, const Blk &b) { return a.cost > b.cost; });
    // every XCD ends with lo or lo + 1 blocks, exactly `extra` of them with lo + 1
    const size_t lo = blk.size() / 8, extra = blk.size() % 8;
    size_t n_plus = 0;
    uint64_t load[8] = {0};
    size_t count[8] = {0};
    lists.assign(8, {});
    for (const Blk &b : blk) {
        int best = -1;
        for (int x8 = 0; x8 < 8; x8++) {
            const bool room = count[x8] < lo || (count[x8] == lo && n_plus < extra);
            if (room && (best < 0 || load[x8] < load[best])) best = x8;
        }
        n_plus += count[best] == lo;
        load[best] += b.cost;
        count[best]++;
        for (uint32_t y = b.j * by; y < std::min(ty, b.j * by + by); y++)
            for (uint32_t x = b.i * bx; x < std::min(tx, b.i * bx + bx); x++)
                lists[best].push_back(y * tx + x);
    }
}

int frame_order(const vr_render_desc *d, uint32_t tx, uint32_t ty, const uint32_t *&perm,
                uint32_t **record) {
    uint32_t bx = 1, by = 4;
    if (const char *e = vr::tuning("VR_XBLOCK")) {
        char *end = nullptr;
        const long a = std::strtol(e, &end, 10);
        long b = a;
        if (end && *end == ',') b = std::strtol(end + 1, nullptr, 10);
        if (a <= 0 || b <= 0) { perm = nullptr; return VR_OK; }
        bx = (uint32_t)std::min(a, 64L);
        by = (uint32_t)std::min(b, 64L);
    }
    // everything that changes the samples each ray takes keys the order
    uint32_t key[22] = {d->width, d->height, bx, by};
    std::memcpy(key + 4, d->inv_view, sizeof d->inv_view);
    key[16] = vr::tuning("VR_NO_LPT") ? 1u : 0u;
    key[17] = (uint32_t)d->query_method;
    std::memcpy(key + 18, &d->density, sizeof(float));
    std::memcpy(key + 19, &d->transfer_offset, sizeof(float));
    std::memcpy(key + 20, &d->transfer_scale, sizeof(float));
    key[21] = g.volume_epoch;
    const size_t ntile = (size_t)tx * ty;
    if (g.perm && std::memcmp(key, g.perm_key, sizeof key) == 0) {
        perm = g.perm;
        if (g.order_state == 1 && record) {
            if (!g.cost_recorded) {  // no frame of this view has recorded yet
                VR_HIP(hipMemsetAsync(g.tile_cost, 0, ntile * sizeof(uint32_t), g.stream));
                *record = g.tile_cost;
                return VR_OK;
            }
            // the frame after the recording one: re-deal the tiles by the costs
            std::vector<uint32_t> cost(ntile);
            VR_HIP(hipMemcpyAsync(cost.data(), g.tile_cost, ntile * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, g.stream));
            VR_HIP(hipStreamSynchronize(g.stream));
            g.order_state = 2;
            bool any = false;
            for (uint32_t c : cost) any |= c != 0;
            if (any) {  // kernels other than the per-ray pipelined march record nothing
                std::vector<std::vector<uint32_t>> lists;
                lists_from_costs(cost, tx, ty, bx, by, lists);
                int rc = upload_perm(lists);
                if (rc != VR_OK) return rc;
                perm = g.perm;
            }
        }
        return VR_OK;
    }
    const uint32_t nbx = (tx + bx - 1) / bx, nby = (ty + by - 1) / by;
    struct Blk { float cost; uint32_t i, j; };
    std::vector<std::vector<Blk>> blocks(8);
    for (uint32_t byi = 0; byi < nby; byi++) {
        for (uint32_t bxi = 0; bxi < nbx; bxi++) {
            float c = 0.0f;
            for (uint32_t y = byi * by; y < std::min(ty, byi * by + by); y++)
                for (uint32_t x = bxi * bx; x < std::min(tx, bxi * bx + bx); x++)
                    for (int k = 0; k < 3; k++)
                        c = std::max(c, est_steps(d->inv_view, d->width, d->height,
                                                  (float)(x * vr::kTileW + k * (vr::kTileW - 1) / 2),
                                                  (float)(y * vr::kTileH + vr::kTileH / 2)));
            blocks[(bxi + 3 * byi) & 7].push_back({c, bxi, byi});
        }
    }
    std::vector<std::vector<uint32_t>> lists(8);
    for (int x8 = 0; x8 < 8; x8++) {
        std::vector<Blk> &bl = blocks[x8];
        if (!key[16])
            std::stable_sort(bl.begin(), bl.end(),
                             [](const Blk &a, const Blk &b) { return a.cost > b.cost; });
        for (const Blk &b : bl)
            for (uint32_t y = b.j * by; y < std::min(ty, b.j * by + by); y++)
                for (uint32_t x = b.i * bx; x < std::min(tx, b.i * bx + bx); x++)
                    lists[x8].push_back(y * tx + x);
    }
    g.order_state = 0;  // until the new order is in place
    int rc = upload_perm(lists);
    if (rc != VR_OK) return rc;
    std::memcpy(g.perm_key, key, sizeof key);
    perm = g.perm;
    g.order_state = (key[16] || vr::tuning("VR_NO_ADAPT")) ? 2 : 1;
    g.cost_recorded = false;
    if (g.order_state == 1) {
        if (ntile > g.tile_cost_cap) {
            if (g.tile_cost) (void)hipFree(g.tile_cost);
            g.tile_cost = nullptr;
            g.tile_cost_cap = 0;
            VR_HIP(hipMalloc(&g.tile_cost, ntile * sizeof(uint32_t)));
            g.tile_cost_cap = ntile;
        }
        if (record) {
            VR_HIP(hipMemsetAsync(g.tile_cost, 0, ntile * sizeof(uint32_t), g.stream));
            *record = g.tile_cost;
        }
    }
    return VR_OK;
}

// LDS bytes per CU and per workgroup of the current device (160 KiB each on
// gfx950), read once per device; the occupancy caps are sized from them
// (vr_march.h cap_lds).
void device_lds(int &per_cu, int &per_wg) {
    static int cached_dev = -1, cu = 160 * 1024, wg = 64 * 1024;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev != cached_dev) {
        int a = 0, b = 0;
        if (hipDeviceGetAttribute(&a, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) ==
                hipSuccess && a > 0)
            cu = a;
        if (hipDeviceGetAttribute(&b, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) ==
                hipSuccess && b > 0)
            wg = b;
        cached_dev = dev;
    }
    per_cu = cu;
    per_wg = wg;
}

// gather8's 32-bit addressing of a baked plane: pitches and depth fit 24-bit
// multiplies and the byte offset of every element fits 32 bits (a 1024^3 plane,
// 2^30 floats, does: the last element sits at 2^32 - 4)
// a baked plane's index fits the 32-bit form of gather8 (MODE 1: 24-bit
// multiplies, 32-bit sums): pitches and depth < 2^24, plane < 2^32 floats
int plane_narrow(uint64_t sy, uint64_t sz, uint64_t nz) {
    return sy < (1u << 24) && sz < (1u << 24) && nz < (1u << 24) && sz * nz < (1ull << 32);
}

int fill_params(const vr_render_desc *d, vr::Params &P, uint32_t &nslots,
                bool for_render = false) {
    if (!d) return fail(VR_ERR_ARG, "null render descriptor");
    const bool codec = d->query_method >= 4 && d->query_method <= 6;
    if (codec && !g.cb)
        return fail(VR_ERR_STATE, "queryMethod %d needs a codec volume (initCuda's codebook / "
                                  "vr_init_codec)", d->query_method);
    const bool flex = is_flex_method(d->query_method);
    if (!codec && !flex && !g.vol)
        return fail(VR_ERR_STATE, "no volume resident (initCuda / vr_init_* first)");
    if (!d->d_output) return fail(VR_ERR_ARG, "d_output is null");
    if (d->width == 0 || d->height == 0) return fail(VR_ERR_ARG, "empty image");
    int rc = check_method(d->query_method);
    if (rc != VR_OK) return rc;
    if (d->query_method == 7 &&
        (d->volume_size.width == 0 || d->volume_size.height == 0 || d->volume_size.depth == 0))
        return fail(VR_ERR_ARG, "method 7 needs a non-empty volumeSize");
    std::memset(&P, 0, sizeof P);
    std::memcpy(P.m, d->inv_view, sizeof P.m);
    P.W = d->width;
    P.H = d->height;
    P.CW = d->width;
    P.CH = d->height;
    P.density = d->density;
    P.brightness = d->brightness;
    P.toff = d->transfer_offset;
    P.tscale = d->transfer_scale;
    if (codec) {  // the codec volume: dense voxel order, its own bin count
        P.nx = g.cnx; P.ny = g.cny; P.nz = g.cnz;
        P.sy = (uint64_t)g.cnx;
        P.sz = (uint64_t)g.cnx * (uint64_t)g.cny;
        P.nb = g.cnb;
        P.cb = g.cb;
        P.tpl = g.tpl;
        P.err = g.cerr;
        P.ntpl = g.ntpl;
        P.err_slots = g.err_slots;
        // template tables up to 32 KiB are staged in LDS (VR_CODEC_LDS=0 disables)
        const size_t tb = (size_t)g.ntpl * g.cnb * sizeof(float);
        const char *el = vr::tuning("VR_CODEC_LDS");
        P.tpl_lds = (tb <= 32768 && !(el && std::atoi(el) == 0)) ? (int)tb : 0;
    } else {
        P.nx = g.nx; P.ny = g.ny; P.nz = g.nz;
        P.sy = g.sy; P.sz = g.sz;
        P.nb = g.nb;
    }
    if (flex) {
        P.flex = g.flex.blocks;
        P.nflex = g.flex.nblk;
        P.nb = g.flex.nb;
    }
    P.m7x = (int)d->volume_size.width;
    P.m7y = (int)d->volume_size.height;
    P.m7z = (int)d->volume_size.depth;
    P.enorm = entropy_norm(P.nb);
    P.tiles_x = tiles_x(d->width);
    P.tile_list = d->d_tile_list;
    P.perm = nullptr;
    uint32_t *record = nullptr;
    if (!d->d_tile_list) {
        int rc = frame_order(d, tiles_x(d->width), tiles_y(d->height), P.perm,
                             for_render ? &record : nullptr);
        if (rc != VR_OK) return rc;
    }
    P.out = d->d_output;
    P.out_f = d->d_output_f;
    P.out_n = d->d_steps;
    P.mark = nullptr;
    // VR_BOX_MAX: per-wave LDS box capacity (tuning / ablation knob; 0 disables staging)
    P.box_max = vr::kBoxMax;
    if (const char *e = vr::tuning("VR_BOX_MAX")) {
        const int v = std::atoi(e);
        if (v >= 0 && v <= 2048) P.box_max = v;
    }
    // VR_WG_PER_CU: cap resident workgroups per CU through the LDS request (tuning knob)
    P.wg_per_cu = 0;
    if (const char *e = vr::tuning("VR_WG_PER_CU")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= 32) P.wg_per_cu = v;
    }
    // Kernel choice (measured at 1024^3 x 8).  When the
    // screen x axis runs along the volume's voxel rows (|m[0]| ~ 1, e.g. the
    // runSingleTest view) consecutive lanes read consecutive records and the
    // per-ray pipelined march (path 2) is fastest for mean and variance; the
    // log-heavy entropy decode prefers the wave-staged march (path 4), which
    // decodes every record once per wave-step instead of once per touching
    // ray.  Oblique views use the quad-cooperative gathers (path 0, B == 8),
    // which keep every 4-lane group on one contiguous 64-byte run.
    // VR_PATH overrides (vr_set_tuning): 0 quad, 1 k_march (LDS-staged box /
    // per-ray), 2 per-ray pipelined, 4 wave-staged rows, 7 ray-segmented
    // (VR_SEG lanes per ray).
    const bool along_rows = std::fabs(d->inv_view[0]) >= 0.95f;
    // (entropy of 1-4 bins: the one-lane pipelined march, round 6 -- 1024^3 x 2
    // 1080p C0 4.66 -> 3.25 ms, x 4 4.51 -> 4.35 against the wave-staged march;
    // profiles/r06/knobs/m3_1024x*.log)
    P.path = along_rows ? (d->query_method == 3 && g.nb >= 8 ? 4 : 2) : 0;
    // 8-bin entropy of row-aligned views: the LDS-box march with the rolled
    // LDS-column entropy (k_march<8,3>, 128 VGPRs) beats the wave-staged march:
    // 1024^3 C0 4.31 -> 3.52 ms, 512^3 3.10 -> 1.63 (round 4,
    // profiles/r04/variants_1024x8_m3.log, variants_512x8_m3.log).  Rank tile
    // lists too: cost-dealt 1024^3 C0 lists, max over ranks, k_march vs the
    // wave-staged march N = 2 1.99 vs 2.52 ms, N = 4 1.52 vs 1.67, N = 8 1.51 vs
    // 1.51 (round 5, profiles/r05/rank_sim_m3_C0_paths.log)
    if (along_rows && d->query_method == 3 && g.nb == 8) P.path = 1;
    // ... and of oblique views of a volume coarse for the frame (>= 4 pixels per
    // voxel of the x-y face): 512^3 C1 m3 8.32 -> 5.11 ms; at 1024^3 the quad
    // march stays ahead (8.42 vs 8.61; profiles/r04/variants_*_m3_r4g.log)
    // (16 and 32 bins too, round 6: 512^3 x 16 C1 m3 8.60 -> 5.56 ms, x 32 15.9 ->
    // 10.3; at 1024^3 the quad march stays ahead, 9.05 vs 10.3 and 16.9 vs 19.1;
    // profiles/r06/knobs/wide_*.log, m3_512x32.log)
    if (!along_rows && d->query_method == 3 && (g.nb == 8 || g.nb == 16 || g.nb == 32) &&
        !d->d_tile_list &&
        (uint64_t)d->width * d->height >= 4ull * (uint64_t)g.nx * (uint64_t)g.ny)
        P.path = 1;
    P.oblique = along_rows ? 0 : 1;
    device_lds(P.lds_cu, P.lds_wg);
    // Views whose screen x runs along the volume's z or y (|M[8]| / |M[4]| >=
    // 0.95) march an axis-rows copy of an owned B <= 8 volume with the per-ray
    // pipelined march (ensure_axis_copy); for the choices below
    // they count as row-aligned (their x-row seg / quad alternatives read the
    // x rows across).  VR_ZROWS=0 keeps them oblique.
    // 8-bin entropy of such views takes the LDS-box march on the x rows instead:
    // the pipelined march decodes all 8 corners' 64 logarithms per step
    // unrolled and spills (1024^3 x 8 side view S m3: 18.8 ms; box 3.38, quad
    // 5.55, wave-staged 5.12; profiles/r06/knobs/side_m3.log)
    const bool axis_dir = std::fabs(d->inv_view[8]) >= 0.95f || std::fabs(d->inv_view[4]) >= 0.95f;
    const bool axis_m3 = !along_rows && axis_dir && d->query_method == 3 && g.nb == 8;
    const char *ez = vr::tuning("VR_ZROWS");
    P.axis_view = 0;
    if (!along_rows && !codec && !flex && g.owned && d->query_method >= 1 &&
        d->query_method <= 3 && (g.nb == 1 || g.nb == 2 || g.nb == 4 || g.nb == 8) &&
        !axis_m3 && !(ez && std::atoi(ez) == 0))
        P.axis_view = std::fabs(d->inv_view[8]) >= 0.95f ? 2 : std::fabs(d->inv_view[4]) >= 0.95f ? 1 : 0;
    const bool row_like = along_rows || P.axis_view != 0;
    if (P.axis_view) P.path = 2;
    if (axis_m3 && !codec && !flex) P.path = 1;
    // Side and top views of 16- and 32-bin records (no axis copy: B <= 8 only)
    // likewise take the LDS-box march on the x rows instead of the quad march:
    // 1024^3 x 32 side view m1 13.7 -> 6.9 ms, m3 15.4 -> 7.6, top view m1 7.6 ->
    // 7.0, m3 15.4 -> 7.5; 1024^3 x 16 side m1 6.7 -> 4.9, m3 8.6 -> 4.4; 512^3 x
    // 16 side m1 3.7 -> 1.3, m3 8.2 -> 1.9 (profiles/r06/knobs/wide_*.log)
    if (!along_rows && axis_dir && (g.nb == 16 || g.nb == 32) && !d->d_tile_list &&
        d->query_method >= 1 && d->query_method <= 3 && !codec && !flex)
        P.path = 1;
    // Launches of few rays (a rank's tile list at 4 or 8 GPUs, 1080p) are bound
    // by the per-ray step chain, not by HBM: there the pipelined ray-segmented
    // march (2 lanes per ray, next window gathered before this one decodes,
    // path 7) renders mean / variance row-aligned views faster than the
    // one-lane march (cost-dealt 1024^3x8 C0 lists, max over ranks: N = 8
    // 0.217 ms vs 0.265 for plain 4-lane windows, N = 4 0.410 vs 0.44 one-lane);
    // at 2 GPUs (~1.04 M rays per rank) the one-lane march still wins (0.70 vs
    // 0.81 ms) (tools/rank_sim.py, tools/gpu_seg4.sh).
    // VR_SEG_RAYS overrides the ray-count threshold.
    uint64_t seg_rays = 700000;
    if (const char *e = vr::tuning("VR_SEG_RAYS")) seg_rays = std::strtoull(e, nullptr, 10);
    // Views along the volume's z or y (axis-rows copy) split the rays of such
    // lists the same way, the windows' gathers addressed in the copy
    // (k_march_segp2_zrows: cost-dealt side-view 1024^3 x 8 lists, max over
    // ranks, N = 8 0.399 -> 0.247 ms, N = 4 0.543 -> 0.445; the one-lane march's
    // step chain bound them; profiles/r03/rank_sim_1024x8_S*.log).
    if (row_like && d->d_tile_list && (d->query_method == 1 || d->query_method == 2) &&
        (uint64_t)d->n_tiles * vr::kTileW * vr::kTileH <= seg_rays)
        P.path = 7;
    // Oblique views of a volume coarse for the frame (>= 4 pixels per voxel of
    // the x-y face, e.g. 512^3 at 1080p): neighbouring rays share most records,
    // the launch is bound by the per-ray step chain rather than HBM, and the
    // pipelined 2-lane segmented march beats the quad march (512^3 x 8 C1: m1
    // 2.05 -> 1.77 ms, m2 1.87 -> 1.63; at 1024^3, 2 pixels per voxel, the quad
    // march stays ahead: 3.49 vs 5.23 ms; profiles/r02/paths_512x8.log).
    if (!row_like && g.nb == 8 && (d->query_method == 1 || d->query_method == 2) &&
        (uint64_t)d->width * d->height >= 4ull * (uint64_t)g.nx * (uint64_t)g.ny)
        P.path = 7;
    // Row-aligned full frames of such a coarse volume: a wave's 64 rays cover
    // ~16 voxel columns, so staging the wave's footprint box in LDS (path 1,
    // each record fetched and decoded once per wave) beats the one-lane
    // pipelined march (512^3 x 8 C0 1080p: m1 1.00 -> 0.88 ms, m2 1.00 -> 0.73;
    // it loses for entropy, oblique views, 1024^3 and launches of <= 262 K
    // rays: profiles/r02/paths_coarse_rows.log).
    // The same holds for 16- and 32-bin records, whose box rows load through the
    // quad-cooperative gathers (512^3 x 32 C0 1080p m1: box 2.97 ms, quad march
    // 6.04; profiles/r02/wide_records.log), entropy included: decoding each record
    // once per wave is what the log-heavy wide decode needs (VR_BOX3=0: quad march).
    const bool wide3 = (g.nb == 16 || g.nb == 32) && d->query_method == 3 &&
                       !(vr::tuning("VR_BOX3") && std::atoi(vr::tuning("VR_BOX3")) == 0);
    // 8-bin mean and variance there take two samples per footprint box
    // (k_march_duo): 512^3 x 8 C0 m1 0.694 -> 0.623 ms, m2 0.571 -> 0.496; three
    // or four per box 0.655 / 0.707; at 1024^3 (VR_PATH=1) the doubled boxes lose,
    // 1.69 -> 2.26 (profiles/r04/variants_*_duo_r4l.log)
    // Side and top views of such a coarse volume too, on the x rows without the
    // axis copy (the face across the view is then y-z or x-z): 512^3 x 8 1080p
    // side view m1 1.14 -> 0.74 ms, m2 1.13 -> 0.55; top view m1 1.08 -> 0.75,
    // m2 1.09 -> 0.54 (profiles/r06/knobs/side_512x8_m*.log)
    const uint64_t face = P.axis_view == 2 ? (uint64_t)g.ny * g.nz
                          : P.axis_view == 1 ? (uint64_t)g.nx * g.nz : (uint64_t)g.nx * g.ny;
    if (row_like && !d->d_tile_list && (g.nb == 8 || g.nb == 16 || g.nb == 32) &&
        (d->query_method == 1 || d->query_method == 2 || (wide3 && along_rows)) &&
        (uint64_t)d->width * d->height > seg_rays &&
        (uint64_t)d->width * d->height >= 4ull * face) {
        P.path = 1;
        P.duo = 2;
    }
    // 32-bin records (the reference's own width) are decode-bound at any volume
    // size, and with a 16x4-pixel block per wave the box decodes each record
    // once per wave-step instead of once per touching ray: row-aligned full
    // frames at 1024^3 x 32, 1080p, C0: m1 6.67 -> 6.18 ms, m2 10.42 -> 9.05,
    // m3 41.0 -> 35.0 (16 bins: no gain; profiles/r03/box_map.log)
    if (along_rows && !d->d_tile_list && g.nb == 32 && d->query_method >= 1 &&
        d->query_method <= 3 && (uint64_t)d->width * d->height > seg_rays)
        P.path = 1;
    // 16-bin entropy of row-aligned full frames: the box decodes each record
    // once per wave-step with the rolled LDS-column entropy (round 4): 1024^3 x
    // 16 C0 m3 12.3 -> 5.6 ms; oblique views keep the quad march (13.7 vs 14.0)
    // (profiles/r04/variants_1024x16_m3_r4g.log)
    if (along_rows && !d->d_tile_list && g.nb == 16 && d->query_method == 3 &&
        (uint64_t)d->width * d->height > seg_rays)
        P.path = 1;
    // Mid-size row-aligned full frames of such a coarse volume (more rays than the
    // small-frame threshold below, fewer than the segmented one: BASELINE config 2,
    // 256^3 x 4 at 512^2): a round of 4 waves per SIMD whose per-step overheads
    // dominate, so the box march with four samples per box (k_march_duo) beats the
    // one-lane march for 4 and 8 bins: 256^3 x 4 C0 m1 0.129 -> 0.105 ms, m2 0.104
    // -> 0.076; 256^3 x 8 at 512^2 m1 0.271 -> 0.245, m2 0.240 -> 0.144; 384^3 x 4 at
    // 768^2 m1 0.197 -> 0.198, m2 0.176 -> 0.137; 2 bins lose (m2 0.188 -> 0.213)
    // (profiles/r04/variants_midsize_duo_r4ad.log)
    {
        const uint64_t rays = (uint64_t)d->width * d->height;
        if (along_rows && !d->d_tile_list && !codec && !flex && (g.nb == 4 || g.nb == 8) &&
            (d->query_method == 1 || d->query_method == 2) && rays > 131072 &&
            rays <= seg_rays && rays >= 4ull * (uint64_t)g.nx * (uint64_t)g.ny) {
            P.path = 1;
            P.duo = 4;
        }
    }
    // Small full frames (BASELINE configs 1 and 2: 128^3 x 1 at 256^2, 256^3 x 4
    // at 512^2) cannot fill the GPU with one ray per lane, so the per-ray step
    // chain sets the time, as for a rank's tile list: the pipelined
    // ray-segmented march, 4 lanes per ray up to 128 K rays, else 2.  Measured
    // (profiles/r02/small_frames.log): 128^3 x 1 C0 0.136 -> 0.082 ms, C1
    // 0.180 -> 0.093; 256^3 x 4 C1 0.224 -> 0.147 (its row-aligned view, 262 K
    // rays, takes the box march above).  Oblique views
    // of 8-bin volumes keep the quad march (as for oblique rank lists).
    int small_seg = 0;
    {
        const uint64_t rays = (uint64_t)d->width * d->height;
        const bool nb_ok = g.nb == 1 || g.nb == 2 || g.nb == 4 || (g.nb == 8 && row_like);
        const uint64_t limit = row_like ? std::min<uint64_t>(seg_rays, 131072) : seg_rays;
        if (!d->d_tile_list && !codec && !flex && rays <= limit && nb_ok &&
            (d->query_method == 1 || d->query_method == 2)) {
            P.path = 7;
            // oblique frames up to 400 K rays on 4-lane windows too (round 4, after
            // the unconditional gathers): 256^3 x 4 C1 at 512^2 0.161 -> 0.135 ms
            // (profiles/r04/variants_256x4_r4g.log)
            small_seg = (rays <= 131072 || (!row_like && rays <= 400000)) ? -4 : -2;
        }
        // Entropy of such frames with 1, 2 or 4 bins (round 4): the wave-staged
        // march (row-aligned) and the one-lane march (oblique) lose to 2-lane
        // windows, and row-aligned coarse frames above 128 K rays to the LDS box:
        // 128^3 x 1 at 256^2 C0 1.066 -> 0.481 ms, C1 0.988 -> 0.514; 256^3 x 4 at
        // 512^2 C0 1.600 -> 1.185 (box), C1 2.299 -> 1.707; 256^3 x 2 at 512^2 C0
        // 1.343 -> 0.783 (box), C1 1.113 -> 1.064 (profiles/r04/variants_midsize_m3_r4ag.log)
        // Round 6, after the cheaper exact log: 2 and 4 bins take the one-lane
        // pipelined march instead (256^3 x 4 at 512^2 C0 1.14 -> 0.99 ms, C1 1.66 ->
        // 1.12; 384^3 x 4 at 768^2 C0 1.84 -> 1.54, C1 2.96 -> 1.65; 256^3 x 2 C0
        // 0.76 -> 0.68, C1 1.04 -> 0.90); one bin keeps the 2-lane windows (128^3
        // x 1 C0 0.47 vs 0.51, C1 0.50 vs 0.80; profiles/r06/knobs/m3_*.log)
        if (!d->d_tile_list && !codec && !flex && d->query_method == 3 && !P.axis_view &&
            (g.nb == 1 || g.nb == 2 || g.nb == 4) && rays <= seg_rays) {
            if (g.nb != 1) {
                P.path = 2;
            } else if (along_rows && rays > 131072 && rays >= 4ull * (uint64_t)g.nx * (uint64_t)g.ny) {
                P.path = 1;
            } else {
                P.path = 7;
                small_seg = -2;
            }
        }
    }
    if (P.path != 2 && P.path != 7) P.axis_view = 0;  // 7: the segmented march reads the copy too
    if (const char *e = vr::tuning("VR_DUO")) {  // 0 / 1: one sample per box, 2-4: that many
        const int v = std::atoi(e);
        if (v >= 0 && v <= 4) P.duo = v;
    }
    if (const char *e = vr::tuning("VR_PATH")) {
        const int v = std::atoi(e);
        if (v == 0 || v == 1 || v == 2 || v == 4 || v == 7) {
            P.path = v;
            P.axis_view = 0;  // a forced path reads the x rows
        }
    }
    // The quad march (path 0: oblique views, B = 8, methods 1-3) of a rank's tile
    // list of <= 700 K rays (N >= 4 GPUs at 1080p) takes two lanes per ray
    // (k_march_quad2): such a launch is bound by its longest waves' step chains,
    // which halve.  Cost-dealt 1024^3 x 8 C1 lists, max over ranks: N = 8
    // 0.586 -> 0.455 ms, N = 4 0.955 -> 0.880; N = 2 (1 M rays) 1.64 -> 1.68 and
    // the full frame 3.15 -> 3.35 keep one lane per ray (tools/rank_sim.py,
    // profiles/r03/rank_sim_1024x8_C1_quad2.log).  VR_QUAD2=0/1 overrides.
    P.quad2 = d->d_tile_list && (uint64_t)d->n_tiles * vr::kTileW * vr::kTileH <= 700000u;
    if (const char *e = vr::tuning("VR_QUAD2")) P.quad2 = std::atoi(e) != 0;
    P.wave_clock = g.wave_clock;
    P.box_check = g.box_check;
    P.tile_cost = record;
    P.seg_lanes = small_seg ? small_seg : -2;  // VR_SEG=S: S lanes per ray, negative = pipelined windows
    if (const char *e = vr::tuning("VR_SEG")) {
        const int v = std::atoi(e);
        if (v == 2 || v == 4 || v == -2 || v == -4) P.seg_lanes = v;
    }
    // A wave's rays as a compact pixel block (16 x 4 one lane per ray, (64 / S / 4)
    // x 4 in S-lane windows) instead of a 64- or 64/S-pixel row: its loads touch
    // fewer lines per instruction.  Measured per launch kind (tools/bench_variants.py,
    // tools/rank_sim.py, profiles/r06/segmap/): small full frames on pipelined
    // windows 128^3 x 1 at 256^2 m1 C0 0.075 -> 0.070 ms, C1 0.078 -> 0.077, m3 C0
    // 0.490 -> 0.438 (C1 0.493 vs 0.501: kept as rows), 256^3 x 4 at 512^2 m1 C1
    // 0.143 -> 0.137; row-aligned 2/4-bin entropy on the one-lane march 1024^3 x 2
    // 1080p C0 3.23 -> 3.03, x 4 4.35 -> 4.16 (oblique: 256^3 x 4 C1 1.13 vs 1.22,
    // kept as rows).  Also kept as rows: the 8-bin one-lane march (headline 1.342
    // vs 1.352, side view 1.588 vs 1.628) and the rank lists of records (C0 N = 4
    // 0.376 vs 0.386, N = 8 0.204 vs 0.219).  VR_SEG_MAP=0/1 overrides.
    P.seg_map = (!d->d_tile_list && P.path == 7 && P.seg_lanes < 0 &&
                 (along_rows || d->query_method != 3)) ||
                (P.path == 2 && P.nb <= 4 && d->query_method == 3 && along_rows && !P.axis_view);
    if (const char *e = vr::tuning("VR_SEG_MAP")) P.seg_map = std::atoi(e) != 0;
    // A rank's list at 8 GPUs (<= 400 K rays, 2-lane windows) is bound by the step
    // chains of its longest tiles: its first 64 slots -- the 8 longest tiles of
    // every XCD sublist -- take 4 lanes per ray in the same launch
    // (k_march_seg_head).  Cost-dealt 1024^3 x 8 lists, max over 8 ranks: C0
    // 0.216 -> 0.202 ms (32 / 96 / 128 slots: 0.204 / 0.204 / 0.207; 8 lanes:
    // 0.212), side view 0.254 -> 0.249-0.263; N = 4 lists (~520 K rays) gain
    // nothing (0.380 both) and keep the plain windows
    // (profiles/r04/rank_sim_C0_head.log, rank_sim_S_head.log).
    // VR_HEAD=slots (0 = off), VR_HEAD_SEG=-2/-4/-8, VR_HEAD_TAIL=1 (one-lane
    // tail, k_march_pipe_head) override.
    P.head_slots = 0;
    if (d->d_tile_list && P.path == 7 && P.nb == 8 &&
        (d->query_method == 1 || d->query_method == 2) &&
        (uint64_t)d->n_tiles * vr::kTileW * vr::kTileH <= 400000u)
        P.head_slots = 64;
    P.head_lanes = -4;
    if (const char *e = vr::tuning("VR_HEAD")) P.head_slots = (uint32_t)std::atoi(e) & ~7u;
    if (const char *e = vr::tuning("VR_HEAD_SEG")) P.head_lanes = std::atoi(e);
    P.head_tail = 0;
    if (const char *e = vr::tuning("VR_HEAD_TAIL")) P.head_tail = std::atoi(e);
    if (!d->d_tile_list) P.head_slots = 0;
    const uint64_t all = (uint64_t)tiles_x(d->width) * tiles_y(d->height);
    if (d->d_tile_list) {
        nslots = d->n_tiles;
    } else {
        if (all > 0xFFFFFFFFull) return fail(VR_ERR_ARG, "image too large");
        nslots = (uint32_t)all;
    }
    P.n_tiles = nslots;
    return VR_OK;
}

// Kernel of a baked-statistics frame (measured at 512^3 and 1024^3 x 8, 1080p,
// profiles/r02/baked_paths.log).  A baked step is a few dozen VALU operations
// and 4 pair loads, so the frame is bound by gather issue and line traffic,
// not by decode: row-aligned views take the one-lane pipelined march (path 2,
// 1024^3 C0 0.375 ms); oblique views, whose lanes' loads touch many lines per
// instruction, split each ray over 4 lanes (path 7, VR_SEG 4: 1024^3 C1 2.02
// -> 1.32 ms, 1.11 at 4 workgroups per CU).  A deeper look-ahead ring (2-8 steps in flight per lane) was
// slower everywhere but 512^3 C1 (within 3 %).  VR_PATH (2 / 7) overrides;
// P.seg_lanes keeps a VR_SEG setting.
int baked_path(const vr_render_desc *d, vr::Params &P) {
    // a plane's axis copy (P.plane_axis 1 / 2) makes a side / top view row-aligned
    const bool along_rows = std::fabs(d->inv_view[0]) >= 0.95f || P.plane_axis == 1 ||
                            P.plane_axis == 2;
    int path = along_rows ? 2 : 7;
    int seg = 4;
    // A rank's tile list (multi-GPU) has few rays, so its longest step chains
    // set the time: row-aligned lists split rays too (cost-dealt 1024^3 C0
    // lists, max over ranks: N = 4 (~520 K rays) pipelined 2-lane windows
    // 0.149 ms vs 0.185 one-lane, N = 8 (~260 K) 4 lanes 0.105 vs 0.165;
    // N = 2 stays one-lane, 0.233 vs 0.281; tools/rank_sim.py --baked).
    if (along_rows && d->d_tile_list) {
        const uint64_t rays = (uint64_t)d->n_tiles * vr::kTileW * vr::kTileH;
        if (rays <= 400000) path = 7;
        else if (rays <= 700000) path = 7, seg = -2;
    }
    if (path == 7 && !vr::tuning("VR_SEG")) P.seg_lanes = seg;
    // compact pixel blocks per wave (fill_params): baked frames gain everywhere
    // but on row-aligned 4-lane windows (1024^3 x 8 1080p C1 0.844 -> 0.817 ms,
    // C0 one-lane 0.310 -> 0.295; rank lists C1 N = 8 0.168 -> 0.153, C0 N = 4
    // 0.133 -> 0.124, C0 N = 8 4-lane 0.093 vs 0.096; profiles/r06/segmap/)
    P.seg_map = !(along_rows && path == 7 && P.seg_lanes > 0);
    // oblique full frames of a fine volume (< 4 pixels per voxel of the x-y
    // face): 4 workgroups per CU, fewer rays' lines in flight per L2 (1024^3
    // C1 1.28 -> 1.11 ms; 2-3 per CU 1.25, 6 1.19); coarse volumes (512^3:
    // 0.67 uncapped vs 0.73) and row-aligned views run uncapped
    if (!along_rows && !d->d_tile_list && P.wg_per_cu == 0 &&
        (uint64_t)d->width * d->height < 4ull * (uint64_t)P.nx * (uint64_t)P.ny)
        P.wg_per_cu = 4;
    if (const char *e = vr::tuning("VR_SEG_MAP")) P.seg_map = std::atoi(e) != 0;
    if (const char *e = vr::tuning("VR_PATH")) {  // the LDS-box march (1) reads x rows only
        const int v = std::atoi(e);
        if (v == 2 || v == 7) path = v;
    }
    return path;
}

// Bakes the statistics planes of the resident raw and codec volumes (whichever
// are resident and not yet baked).  On an allocation failure nothing changes:
// the march keeps decoding records per step.
int bake_stats() {
    if (!g.vol && !g.cb) return fail(VR_ERR_STATE, "no volume resident (initCuda / vr_init_* first)");
    vr::Params P;
    std::memset(&P, 0, sizeof P);
    if (g.vol && !g.stats) {
        P.nx = g.nx; P.ny = g.ny; P.nz = g.nz;
        P.sy = g.sy; P.sz = g.sz;
        P.nb = g.nb;
        P.enorm = entropy_norm(g.nb);
        uint64_t psy = 0, psz = 0;
        vr::plane_pitches((uint32_t)g.nx, (uint32_t)g.ny, psy, psz);
        const uint64_t plane = psz * (uint64_t)g.nz;
        float *buf = nullptr;
        VR_HIP(hipMalloc(&buf, (4 * plane + 4) * sizeof(float)));
        hipError_t e = hipMemsetAsync(buf, 0, (4 * plane + 4) * sizeof(float), g.stream);
        if (e == hipSuccess) e = vr::launch_bake_raw(g.vol, P, buf, plane, psy, psz, g.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
        if (e != hipSuccess) {
            (void)hipFree(buf);
            return hip_fail(e, "basicDataProcessing(k_bake_raw)");
        }
        g.stats = buf;
        g.stats_plane = plane;
        g.stats_sy = psy;
        g.stats_sz = psz;
    }
    if (g.cb && !g.cstats) {
        std::memset(&P, 0, sizeof P);
        P.nx = g.cnx; P.ny = g.cny; P.nz = g.cnz;
        P.sy = (uint64_t)g.cnx;
        P.sz = (uint64_t)g.cnx * (uint64_t)g.cny;
        P.nb = g.cnb;
        P.enorm = entropy_norm(g.cnb);
        P.cb = g.cb;
        P.tpl = g.tpl;
        P.err = g.cerr;
        P.ntpl = g.ntpl;
        P.err_slots = g.err_slots;
        uint64_t psy = 0, psz = 0;
        vr::plane_pitches((uint32_t)g.cnx, (uint32_t)g.cny, psy, psz);
        const uint64_t plane = psz * (uint64_t)g.cnz;
        float *buf = nullptr;
        VR_HIP(hipMalloc(&buf, (3 * plane + 4) * sizeof(float)));
        hipError_t e = hipMemsetAsync(buf, 0, (3 * plane + 4) * sizeof(float), g.stream);
        if (e == hipSuccess) e = vr::launch_bake_codec(P, buf, plane, psy, psz, g.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
        if (e != hipSuccess) {
            (void)hipFree(buf);
            if (e == hipErrorInvalidValue)
                return fail(VR_ERR_UNSUPPORTED, "baking codec volumes with %d bins", g.cnb);
            return hip_fail(e, "basicDataProcessing(k_bake_codec)");
        }
        g.cstats = buf;
        g.cstats_plane = plane;
        g.cstats_sy = psy;
        g.cstats_sz = psz;
    }
    return VR_OK;
}

// ---- synthetic volume tables ----
uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

void blob_axis(int n, double c, double s, float *out) {
    for (int i = 0; i < n; i++) {
        const double q = ((double)i + 0.5) / (double)n;
        out[i] = (float)std::exp(-(q - c) * (q - c) / (2.0 * s * s));
    }
}

// Oblique views of an 8-bin volume (the quad march, path 0) read a 2x2 (x, y)
// micro-brick copy of the records: a footprint's four (x, y) corners share
// one 128-B line when x0 and y0 are even, so a wave step touches fewer lines
// than in x rows.  Made on the first such frame of an owned
// volume (a caller-owned buffer adopted by vr_init_distribution may change
// behind the library's back), only if HBM keeps max(4 GiB, 5 %) free after it; without
// it the quad march reads the x rows.  VR_BRICK=0 (vr_set_tuning) disables it.
bool ensure_brick() {
    if (const char *e = vr::tuning("VR_BRICK"))
        if (std::atoi(e) == 0) return false;
    if (g.brick) return true;
    if (!g.vol || !g.owned || g.nb != 8) return false;
    const uint64_t nxp = (uint64_t)g.nx + (g.nx & 1), nyp = (uint64_t)g.ny + (g.ny & 1);
    const uint64_t bsy = 2 * nxp, bsz = nxp * nyp;
    const uint64_t bytes = bsz * (uint64_t)g.nz * 8 * sizeof(float);
    if (!layout_room(bytes)) return false;
    float *buf = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    vr::Params P;
    std::memset(&P, 0, sizeof P);
    P.nx = g.nx; P.ny = g.ny; P.nz = g.nz;
    P.sy = g.sy; P.sz = g.sz;
    // synchronous, like the statistics bake: a later frame may run on another
    // stream (vr_set_stream) and must never see a partly written copy
    const auto t0 = std::chrono::steady_clock::now();
    if (vr::launch_brick8(g.vol, P, buf, bsy, bsz, g.stream) != hipSuccess ||
        hipStreamSynchronize(g.stream) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(buf);
        return false;
    }
    g.layout_last_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.layout_last_bytes = bytes;
    g.layout_builds++;
    g.brick = buf;
    g.bsy = bsy;
    g.bsz = bsz;
    g.brick_bytes = bytes;
    return true;
}

// Views whose screen x runs along the volume's z or y axis (|M[8]| or |M[4]|
// >= 0.95: side views, e.g. the display() camera at yaw 90 deg, and top views
// at pitch and yaw 90 deg) see the x rows across: a wave's 64 rays sit at
// consecutive z (y), each reading its own lines.  A copy of the records with
// that axis contiguous (axis_copy_strides) gives them what x rows give the
// runSingleTest view -- consecutive lanes on consecutive records -- and the
// per-ray pipelined march reads it (1024^3 x 8, yaw 90: 3.01 -> 1.63 ms,
// DESIGN.md 2).  Both axis copies stay resident when the layout budget holds
// them (vr_set_layout_budget); otherwise a view along the other axis replaces
// the copy.  Made on the first such frame of an owned volume with B <= 8 (as
// ensure_brick: synchronous, timed into vr_layout_info) by k_axis_copy, an
// LDS-tiled transpose; VR_ZROWS=0 (vr_set_tuning) disables it.
bool ensure_axis_copy(int axis) {
    if (const char *e = vr::tuning("VR_ZROWS"))
        if (std::atoi(e) == 0) return false;
    const int i = axis - 1, other = 1 - i;
    if (g.acopy[i].buf) return true;
    if (!g.vol || !g.owned || !(g.nb == 1 || g.nb == 2 || g.nb == 4 || g.nb == 8)) return false;
    uint64_t sx = 0, sy = 0, sz = 0;
    vr::axis_copy_strides(axis, (uint64_t)g.nx, (uint64_t)g.ny, (uint64_t)g.nz, sx, sy, sz);
    const uint64_t bytes = (uint64_t)g.nx * g.ny * (uint64_t)g.nz * (uint64_t)g.nb * sizeof(float);
    // keep the other axis' copy when both fit; drop it only if that makes room
    // (checked before anything is released)
    if (!layout_room(bytes)) {
        if (!g.acopy[other].buf || !layout_room(bytes, g.acopy[other].bytes)) return false;
        release_axis_copy(other);
    }
    float *buf = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    vr::Params P;
    std::memset(&P, 0, sizeof P);
    P.nx = g.nx; P.ny = g.ny; P.nz = g.nz; P.nb = g.nb;
    P.sy = g.sy; P.sz = g.sz;
    const auto t0 = std::chrono::steady_clock::now();
    if (vr::launch_axis_copy(g.vol, P, buf, sx, sy, sz, g.stream) != hipSuccess ||
        hipStreamSynchronize(g.stream) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(buf);
        return false;
    }
    g.layout_last_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.layout_last_bytes = bytes;
    g.layout_builds++;
    g.acopy[i].buf = buf;
    g.acopy[i].sx = sx;
    g.acopy[i].sy = sy;
    g.acopy[i].sz = sz;
    g.acopy[i].bytes = bytes;
    return true;
}

// Baked frames of views whose screen x runs along the volume's y or z (side
// and top views) read the planes' 16 x 2 x 1 bricks across: a wave's 64 rays
// sit at consecutive z (y), each on its own lines.  The plane the method
// filters gets a copy with that axis in the brick rows (k_plane_axis), the
// axis-rows idea of ensure_axis_copy for planes: one per axis, made on the
// first such frame within the layout budget, dropped with the planes.
// Axis 3 (round 5): oblique views get the plane in 8 x 2 x 2 bricks
// (k_plane8, gather8 MODE 6), whose lines also hold a footprint's z pair
// (per 64x4-tile line floor at 1024^3 C1: 3.77 -> 3.47 GB);
// VR_PLANE8=0 keeps such views on the 16 x 2 x 1 plane.
// Each (axis, method plane) keeps its own copy while the layout budget holds
// them, so a client alternating methods on one view class builds each copy
// once (one copy per axis was rebuilt -- hipMalloc, k_plane8, a
// stream sync, ~4.6 GB at 1024^3 -- on every method change); only when the
// budget is short are this axis' other planes' copies dropped for the new one.
bool ensure_plane_copy(int plane, int axis) {
    if (const char *e = vr::tuning(axis == 3 ? "VR_PLANE8" : "VR_ZROWS"))
        if (std::atoi(e) == 0) return false;
    const int i = axis - 1;
    if (!g.stats || plane < 0 || plane > 2) return false;
    if (g.pcopy[i][plane].buf) return true;
    const uint32_t nf = axis == 2 ? g.nz : g.ny, np = axis == 2 ? g.ny : g.nx;
    uint64_t ns = axis == 2 ? (uint64_t)g.nx : (uint64_t)g.nz;
    if (nf >= (1u << 16) || np > 65535 || ns > 65535 || g.nx > 65535) return false;
    uint64_t dsy = 0, dsz = 0;
    if (axis == 3) {
        vr::plane8_pitches(g.nx, g.ny, dsy, dsz);
        ns = (uint64_t)(g.nz + 1) / 2;  // slice pairs
    } else {
        vr::plane_pitches(nf, np, dsy, dsz);
    }
    // gather8 MODE 4/5/6: 32-bit offsets inside a slice (pair)
    if (dsz >= (1ull << 32)) return false;
    const uint64_t bytes = (dsz * ns + 4) * sizeof(float);
    if (!layout_room(bytes, 0)) {  // room only without this axis' other planes' copies
        uint64_t freed = 0;
        for (int p = 0; p < 3; p++) freed += g.pcopy[i][p].bytes;
        if (!layout_room(bytes, freed)) return false;
        for (int p = 0; p < 3; p++) release_plane_copy(i, p);
    }
    float *buf = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const float *src = g.stats + (uint64_t)plane * g.stats_plane;
    if (hipMemsetAsync(buf, 0, bytes, g.stream) != hipSuccess ||
        (axis == 3 ? vr::launch_plane8(src, g.stats_sy, g.stats_sz, buf, dsy, dsz, g.nx, g.ny,
                                       g.nz, g.stream)
                   : vr::launch_plane_axis(src, g.stats_sy, g.stats_sz, buf, dsy, dsz, g.nx,
                                           g.ny, g.nz, axis, g.stream)) != hipSuccess ||
        hipStreamSynchronize(g.stream) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(buf);
        return false;
    }
    g.layout_last_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.layout_last_bytes = bytes;
    g.layout_builds++;
    g.pcopy[i][plane].buf = buf;
    g.pcopy[i][plane].sy = dsy;
    g.pcopy[i][plane].sz = dsz;
    g.pcopy[i][plane].bytes = bytes;
    return true;
}

}  // namespace

namespace vr {
int record_error(int status, const char *msg) { return fail(status, "%s", msg); }
const char *tuning(const char *key) {
    auto it = g_tuning.find(key);
    if (it != g_tuning.end()) return it->second.c_str();
#ifdef VR_TUNING
    return std::getenv(key);
#else
    return nullptr;
#endif
}
// Span index: sorted keys and, per key, the entry the reference's linear scan
// (K:1352-1372) returns -- its `break` leaves only the x loop, so among equal
// spans the last 64-entry row holding one wins, and its first entry.  Entries
// with a coordinate outside [0, 1023] can never match a sub-span and are left out.
void build_span_index(const vr_int4 *lo, const vr_int4 *hi, int n,
                             std::vector<uint64_t> &keys, std::vector<int32_t> &idx) {
    std::vector<std::pair<uint64_t, int32_t>> kv;
    kv.reserve((size_t)n);
    for (int i = 0; i < n; i++) {
        const int c[6] = {lo[i].x, lo[i].y, lo[i].z, hi[i].x, hi[i].y, hi[i].z};
        bool ok = true;
        for (int q = 0; q < 6; q++) ok = ok && c[q] >= 0 && c[q] < 1024;
        if (ok) kv.push_back({vr::span_key(c[0], c[1], c[2], c[3], c[4], c[5]), i});
    }
    std::sort(kv.begin(), kv.end());
    keys.clear();
    idx.clear();
    for (size_t a = 0; a < kv.size();) {
        size_t b = a;
        while (b < kv.size() && kv[b].first == kv[a].first) b++;
        const int32_t last_row = kv[b - 1].second / 64;
        size_t pick = a;
        while (kv[pick].second / 64 != last_row) pick++;
        keys.push_back(kv[a].first);
        idx.push_back(kv[pick].second);
        a = b;
    }
}

template <typename T>
hipError_t upload(T *&dst, const T *src, size_t n) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMalloc(&dst, n * sizeof(T));
    if (e == hipSuccess) e = hipMemcpy(dst, src, n * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

}  // namespace vr

extern "C" {

const char *vr_version(void) { return "vrdd-amd 0.1 (gfx950)"; }

const char *vr_last_kernel(void) { return vr::last_march_kernel(); }

// Measured read ceiling: the resident record volume streamed
// once per rep by k_stream_read on the library's stream, timed with HIP events.
int vr_stream_read(int reps, float *ms, uint64_t *bytes) {
    if (!ms || reps < 1) return fail(VR_ERR_ARG, "vr_stream_read: ms null or reps < 1");
    if (!g.vol) return fail(VR_ERR_STATE, "no volume resident");
    const uint64_t nbytes = (g.sz * (uint64_t)g.nz * (uint64_t)g.nb * 4u) & ~(uint64_t)15;
    hipDevice_t dev;
    int dev_id = 0, cus = 0;
    VR_HIP(hipGetDevice(&dev_id));
    (void)dev;
    VR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id));
    const uint32_t nblocks = (uint32_t)(cus > 0 ? cus : 256) * 8u;  // 8 workgroups per CU
    uint32_t *d = nullptr;
    VR_HIP(hipMalloc(&d, nblocks * sizeof(uint32_t)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    float best = 0.0f, sum = 0.0f;
    // one untimed pass first (clocks, address translation)
    if (e == hipSuccess) e = vr::launch_stream_read(g.vol, nbytes, d, nblocks, g.stream);
    for (int r = 0; r < reps && e == hipSuccess; r++) {
        e = hipEventRecord(e0, g.stream);
        if (e == hipSuccess) e = vr::launch_stream_read(g.vol, nbytes, d, nblocks, g.stream);
        if (e == hipSuccess) e = hipEventRecord(e1, g.stream);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float t = 0.0f;
        if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
        if (e == hipSuccess) {
            best = (r == 0 || t < best) ? t : best;
            sum += t;
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "vr_stream_read");
    ms[0] = best;
    ms[1] = sum / (float)reps;
    if (bytes) *bytes = nbytes;
    return VR_OK;
}

int vr_selftest_logf(uint64_t *counts) {
    if (!counts) return fail(VR_ERR_ARG, "null pointer");
    unsigned long long *d = nullptr;
    VR_HIP(hipMalloc(&d, 2 * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, 2 * sizeof(unsigned long long), g.stream);
    if (e == hipSuccess) e = vr::launch_logcheck(d, g.stream);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, g.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "vr_selftest_logf");
    counts[0] = h[0];
    counts[1] = h[1];
    return VR_OK;
}

const char *vr_last_error(void) { return g.err.c_str(); }
int vr_last_status(void) { return g.status; }
void vr_clear_error(void) {
    g.err.clear();
    g.status = VR_OK;
}

uint32_t vr_tiles_x(uint32_t width) { return tiles_x(width); }
uint32_t vr_tiles_y(uint32_t height) { return tiles_y(height); }

int vr_set_tuning(const char *key, const char *value) {
    if (!key || !*key) return fail(VR_ERR_ARG, "vr_set_tuning: empty key");
    if (value) g_tuning[key] = value;
    else g_tuning.erase(key);
    g.perm_key[0] = 0;  // knobs such as VR_XBLOCK / VR_NO_LPT shape the frame order
    return VR_OK;
}

void vr_clear_tuning(void) {
    g_tuning.clear();
    g.perm_key[0] = 0;
}

int vr_set_stream(void *stream) {
    g.stream = (hipStream_t)stream;
    return VR_OK;
}

int vr_init_codec(const vr_int4 *codebook, vr_extent dims, const float *templates,
                  int ntemplates, const vr_float2 *errors, int err_slots, int nbins, int where) {
    if (!codebook || !templates || (!errors && err_slots > 0))
        return fail(VR_ERR_ARG, "vr_init_codec: null array");
    if (where != 0 && where != 1) return fail(VR_ERR_ARG, "vr_init_codec: where must be 0 or 1");
    if (dims.width == 0 || dims.height == 0 || dims.depth == 0 || nbins <= 0 ||
        ntemplates <= 0 || err_slots < 0 || dims.width > 65535 || dims.height > 65535 ||
        dims.depth > 65535)
        return fail(VR_ERR_ARG, "vr_init_codec: bad sizes");
    if (nbins != 1 && nbins != 2 && nbins != 4 && nbins != 8 && nbins != 16 && nbins != 32)
        return fail(VR_ERR_UNSUPPORTED, "vr_init_codec: %d bins (compiled: 1,2,4,8,16,32)", nbins);
    const uint64_t nvox = (uint64_t)dims.width * dims.height * dims.depth;
    release_codec();
    const hipMemcpyKind kind = where == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    const size_t bcb = nvox * sizeof(int4), btp = (size_t)ntemplates * nbins * sizeof(float);
    const size_t ber = nvox * (size_t)err_slots * sizeof(float2);
    VR_HIP(hipMalloc(&g.cb, bcb));
    VR_HIP(hipMalloc(&g.tpl, btp));
    if (ber) VR_HIP(hipMalloc(&g.cerr, ber));
    hipError_t e = hipMemcpy(g.cb, codebook, bcb, kind);
    if (e == hipSuccess) e = hipMemcpy(g.tpl, templates, btp, kind);
    if (e == hipSuccess && ber) e = hipMemcpy(g.cerr, errors, ber, kind);
    unsigned long long *bad = nullptr, hbad = 0;
    if (e == hipSuccess) e = hipMalloc(&bad, sizeof hbad);
    if (e == hipSuccess) e = hipMemset(bad, 0, sizeof hbad);
    if (e == hipSuccess) e = vr::launch_codec_check(g.cb, nvox, ntemplates, nbins, err_slots, bad, 0);
    if (e == hipSuccess) e = hipMemcpy(&hbad, bad, sizeof hbad, hipMemcpyDeviceToHost);
    if (bad) (void)hipFree(bad);
    if (e != hipSuccess) {
        release_codec();
        return hip_fail(e, "vr_init_codec");
    }
    if (hbad) {
        release_codec();
        return fail(VR_ERR_ARG,
                    "vr_init_codec: %llu codebook entries out of range (template id < %d, "
                    "0 <= shift < %d, 0 <= NE <= %d)", hbad, ntemplates, nbins, err_slots);
    }
    g.cnx = (int)dims.width;
    g.cny = (int)dims.height;
    g.cnz = (int)dims.depth;
    g.cnb = nbins;
    g.ntpl = ntemplates;
    g.err_slots = err_slots;
    return VR_OK;
}

int vr_init_flex(const vr_flex_tables *t) {
    if (!t) return fail(VR_ERR_ARG, "vr_init_flex: null tables");
    if (t->dim < 1 || t->dim > vr::kFlexMaxDim)
        return fail(VR_ERR_ARG, "vr_init_flex: dim %d outside [1, %d]", t->dim, vr::kFlexMaxDim);
    if (t->nbins < 1 || t->nbins > vr::kFlexMaxBins)
        return fail(VR_ERR_ARG, "vr_init_flex: nbins %d outside [1, %d]", t->nbins,
                    vr::kFlexMaxBins);
    if (t->n_fractal < 0 || t->n_simple < 0 || (t->n_fractal > 0 && t->ntemplates < 1))
        return fail(VR_ERR_ARG, "vr_init_flex: bad table sizes");
    if ((t->n_fractal > 0 && (!t->fractal_low || !t->fractal_high || !t->fractal_code ||
                              !t->fractal_errors || !t->templates)) ||
        (t->n_simple > 0 && (!t->simple_low || !t->simple_high || !t->simple_count ||
                             !t->simple_hist)))
        return fail(VR_ERR_ARG, "vr_init_flex: null array");
    const int nb = t->nbins;
    for (int i = 0; i < t->n_fractal; i++) {  // K:1377-1385 (the reference only prints)
        const vr_int4 c = t->fractal_code[i];
        if (c.x < 0 || c.x >= t->ntemplates || c.y < 0 || c.y >= nb || c.w < 0 || c.w > nb)
            return fail(VR_ERR_ARG,
                        "vr_init_flex: fractal entry %d out of range (template %d of %d, shift %d, "
                        "NE %d, %d bins)", i, c.x, t->ntemplates, c.y, c.w, nb);
    }
    for (int i = 0; i < t->n_simple; i++)
        if (t->simple_count[i] < 0 || t->simple_count[i] > nb)
            return fail(VR_ERR_ARG, "vr_init_flex: simple entry %d has %d bins", i,
                        t->simple_count[i]);
    std::vector<uint64_t> fk, sk;
    std::vector<int32_t> fi, si;
    vr::build_span_index(t->fractal_low, t->fractal_high, t->n_fractal, fk, fi);
    vr::build_span_index(t->simple_low, t->simple_high, t->n_simple, sk, si);
    release_flex();
    State::Flex &f = g.flex;
    hipError_t e = vr::upload(f.fkeys, fk.data(), fk.size());
    if (e == hipSuccess) e = vr::upload(f.fidx, fi.data(), fi.size());
    if (e == hipSuccess) e = vr::upload(f.skeys, sk.data(), sk.size());
    if (e == hipSuccess) e = vr::upload(f.sidx, si.data(), si.size());
    if (e == hipSuccess)
        e = vr::upload(f.fcode, reinterpret_cast<const int4 *>(t->fractal_code), (size_t)t->n_fractal);
    if (e == hipSuccess)
        e = vr::upload(f.ferr, reinterpret_cast<const float2 *>(t->fractal_errors),
                   (size_t)t->n_fractal * nb);
    if (e == hipSuccess) e = vr::upload(f.scount, t->simple_count, (size_t)t->n_simple);
    if (e == hipSuccess)
        e = vr::upload(f.shist, reinterpret_cast<const float2 *>(t->simple_hist),
                   (size_t)t->n_simple * nb);
    if (e == hipSuccess && t->n_fractal > 0)
        e = vr::upload(f.tpl, t->templates, (size_t)t->ntemplates * nb);
    if (e != hipSuccess) {
        release_flex();
        return hip_fail(e, "vr_init_flex");
    }
    f.dim = t->dim;
    f.nb = nb;
    f.ntpl = t->ntemplates;
    f.nf = t->n_fractal;
    f.ns = t->n_simple;
    f.nfk = (int)fk.size();
    f.nsk = (int)sk.size();
    return VR_OK;
}

int vr_flex_process(int block) {
    State::Flex &f = g.flex;
    if (f.dim == 0) return fail(VR_ERR_STATE, "vr_flex_process: no span tables (vr_init_flex)");
    if (block < 1 || block > f.dim)
        return fail(VR_ERR_ARG, "vr_flex_process: block %d outside [1, %d]", block, f.dim);
    const int nblk = (f.dim + block - 1) / block;  // K:906-931
    const size_t nblocks = (size_t)nblk * nblk * nblk;
    release_flex_blocks();
    vr::FlexTables T;
    T.dim = f.dim;
    T.nb = f.nb;
    T.fkeys = f.fkeys;
    T.fidx = f.fidx;
    T.nfk = f.nfk;
    T.fcode = f.fcode;
    T.ferr = f.ferr;
    T.skeys = f.skeys;
    T.sidx = f.sidx;
    T.nsk = f.nsk;
    T.scount = f.scount;
    T.shist = f.shist;
    T.tpl = f.tpl;
    float *ch = nullptr;
    unsigned int *missing = nullptr, hmiss = 0;
    float4 *blocks = nullptr;
    hipError_t e = hipMalloc(&ch, nblocks * 8 * f.nb * sizeof(float) + 256);
    if (e == hipSuccess) e = hipMalloc(&blocks, nblocks * sizeof(float4));
    if (e == hipSuccess) {
        missing = reinterpret_cast<unsigned int *>(ch + nblocks * 8 * f.nb);
        e = hipMemsetAsync(missing, 0, sizeof(unsigned int), g.stream);
    }
    if (e == hipSuccess) e = vr::launch_flex_corners(T, block, nblk, ch, missing, g.stream);
    if (e == hipSuccess) e = vr::launch_flex_blocks(f.nb, nblk, ch, blocks, g.stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(&hmiss, missing, sizeof hmiss, hipMemcpyDeviceToHost, g.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    if (ch) (void)hipFree(ch);
    if (e != hipSuccess) {
        if (blocks) (void)hipFree(blocks);
        return hip_fail(e, "vr_flex_process");
    }
    if (hmiss) {
        (void)hipFree(blocks);
        return fail(VR_ERR_ARG, "vr_flex_process: a sub-span of some block corner has no table "
                                "entry (the reference reads an uninitialised codebook entry)");
    }
    f.blocks = blocks;
    f.nblk = nblk;
    return nblk;
}

int vr_flex_info(int *nblk, int *nbins, const float **d_blocks) {
    if (nblk) *nblk = g.flex.nblk;
    if (nbins) *nbins = g.flex.nb;
    if (d_blocks) *d_blocks = reinterpret_cast<const float *>(g.flex.blocks);
    return g.flex.blocks ? VR_OK : fail(VR_ERR_STATE, "no flexible-block statistics resident");
}

int vr_init_distribution(const float *bins, vr_extent dims, int nbins, int where) {
    if (!bins) return fail(VR_ERR_ARG, "null distribution pointer");
    if (nbins < 1) return fail(VR_ERR_ARG, "nbins must be >= 1 (got %d)", nbins);
    if (dims.width == 0 || dims.height == 0 || dims.depth == 0)
        return fail(VR_ERR_ARG, "empty volume");
    if (dims.width > 65536 || dims.height > 65536 || dims.depth > 65536)
        return fail(VR_ERR_ARG, "volume dimension > 65536");
    release_volume();
    const int nx = (int)dims.width, ny = (int)dims.height, nz = (int)dims.depth;
    uint64_t sy, sz;
    if (where == 2) {  // adopted buffer keeps its dense AoS layout
        sy = (uint64_t)nx;
        sz = sy * (uint64_t)ny;
        g.vol = const_cast<float *>(bins);
        g.owned = false;
    } else {
        choose_pitch(nx, ny, sy, sz);
        const size_t rec = (size_t)nbins * sizeof(float);
        float *d = nullptr;
        VR_HIP(hipMalloc(&d, sz * (size_t)nz * rec));
        const hipMemcpyKind kind = where == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
        hipError_t e = hipSuccess;
        if (sy == (uint64_t)nx && sz == sy * (uint64_t)ny) {
            e = hipMemcpy(d, bins, sz * (size_t)nz * rec, kind);
        } else {  // one pitched 2-D copy per slice
            for (int z = 0; z < nz && e == hipSuccess; z++)
                e = hipMemcpy2D(d + (size_t)z * sz * nbins, sy * rec,
                                bins + (size_t)z * ny * nx * nbins, (size_t)nx * rec,
                                (size_t)nx * rec, (size_t)ny, kind);
        }
        if (e != hipSuccess) {
            (void)hipFree(d);
            return hip_fail(e, "hipMemcpy(volume)");
        }
        g.vol = d;
        g.owned = true;
    }
    g.sy = sy;
    g.sz = sz;
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
    g.nb = nbins;
    return VR_OK;
}

// the section-5 blob field tables (host), shared by both synthesizers
void blob_tables(int nx, int ny, int nz, uint64_t seed, vr::SynthArgs &a, std::vector<float> &gx,
                 std::vector<float> &gy, std::vector<float> &gz) {
    gx.assign((size_t)vr::kSynthBlobs * nx, 0.0f);
    gy.assign((size_t)vr::kSynthBlobs * ny, 0.0f);
    gz.assign((size_t)vr::kSynthBlobs * nz, 0.0f);
    for (int k = 0; k < vr::kSynthBlobs; k++) {
        double r[5];
        for (int j = 0; j < 5; j++)
            r[j] = u01(splitmix64(seed + 0x100u + 8u * (uint64_t)k + (uint64_t)j));
        a.amp[k] = (float)(0.3 + 0.7 * r[0]);
        const double s = 0.05 + 0.15 * r[4];
        blob_axis(nx, 0.2 + 0.6 * r[1], s, gx.data() + (size_t)k * nx);
        blob_axis(ny, 0.2 + 0.6 * r[2], s, gy.data() + (size_t)k * ny);
        blob_axis(nz, 0.2 + 0.6 * r[3], s, gz.data() + (size_t)k * nz);
    }
}

int vr_synthesize_codec(vr_extent dims, int nbins, int ntemplates, int slots, uint64_t seed) {
    if (nbins != 1 && nbins != 2 && nbins != 4 && nbins != 8 && nbins != 16 && nbins != 32)
        return fail(VR_ERR_UNSUPPORTED, "codec volumes with %d bins (compiled: 1,2,4,8,16,32)", nbins);
    if (ntemplates < 1 || slots < 0 || slots > nbins)
        return fail(VR_ERR_ARG, "vr_synthesize_codec: bad template count or slots");
    if (dims.width == 0 || dims.height == 0 || dims.depth == 0 || dims.width > 65535 ||
        dims.height > 65535 || dims.depth > 65535)
        return fail(VR_ERR_ARG, "vr_synthesize_codec: bad dims");
    const int nx = (int)dims.width, ny = (int)dims.height, nz = (int)dims.depth;
    const uint64_t nvox = (uint64_t)nx * ny * nz;
    vr::SynthArgs a{};
    std::vector<float> gx, gy, gz;
    blob_tables(nx, ny, nz, seed, a, gx, gy, gz);
    // templates: discretised Gaussians of mean (t + 0.5) / T, sigma 0.06 (double, normalised)
    std::vector<float> tpl((size_t)ntemplates * nbins);
    for (int t = 0; t < ntemplates; t++) {
        const double mu = ((double)t + 0.5) / (double)ntemplates;
        std::vector<double> e(nbins);
        double sum = 0.0;
        for (int b = 0; b < nbins; b++) {
            const double dd = ((double)b + 0.5) / (double)nbins - mu;
            e[b] = std::exp(-dd * dd / (2.0 * 0.06 * 0.06));
            sum += e[b];
        }
        for (int b = 0; b < nbins; b++) tpl[(size_t)t * nbins + b] = (float)(e[b] / sum);
    }
    release_codec();
    float *dgx = nullptr, *dgy = nullptr, *dgz = nullptr;
    hipError_t e = hipMalloc(&g.cb, nvox * sizeof(int4));
    if (e == hipSuccess && slots) e = hipMalloc(&g.cerr, nvox * (size_t)slots * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&g.tpl, tpl.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgx, gx.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgy, gy.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgz, gz.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(g.tpl, tpl.data(), tpl.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgx, gx.data(), gx.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgy, gy.data(), gy.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgz, gz.data(), gz.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        a.gx = dgx; a.gy = dgy; a.gz = dgz;
        a.nx = nx; a.ny = ny; a.nz = nz; a.nb = nbins; a.seed = seed;
        e = vr::launch_synth_codec(g.cb, g.cerr, a, ntemplates, slots, g.stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    if (dgx) (void)hipFree(dgx);
    if (dgy) (void)hipFree(dgy);
    if (dgz) (void)hipFree(dgz);
    if (e != hipSuccess) {
        release_codec();
        return hip_fail(e, "vr_synthesize_codec");
    }
    g.cnx = nx; g.cny = ny; g.cnz = nz; g.cnb = nbins; g.ntpl = ntemplates; g.err_slots = slots;
    return VR_OK;
}

int vr_codec_info(vr_extent *dims, int *nbins, int *ntemplates, int *slots, const void **codebook,
                  const float **templates, const void **errors) {
    if (!g.cb) return fail(VR_ERR_STATE, "no codec volume resident");
    if (dims) {
        dims->width = (size_t)g.cnx;
        dims->height = (size_t)g.cny;
        dims->depth = (size_t)g.cnz;
    }
    if (nbins) *nbins = g.cnb;
    if (ntemplates) *ntemplates = g.ntpl;
    if (slots) *slots = g.err_slots;
    if (codebook) *codebook = g.cb;
    if (templates) *templates = g.tpl;
    if (errors) *errors = g.cerr;
    return VR_OK;
}

int vr_synthesize(vr_extent dims, int nbins, uint64_t seed) {
    if (nbins < 1) return fail(VR_ERR_ARG, "nbins must be >= 1 (got %d)", nbins);
    if (dims.width == 0 || dims.height == 0 || dims.depth == 0)
        return fail(VR_ERR_ARG, "empty volume");
    if (dims.width > 65536 || dims.height > 65536 || dims.depth > 65536)
        return fail(VR_ERR_ARG, "volume dimension > 65536");
    const int nx = (int)dims.width, ny = (int)dims.height, nz = (int)dims.depth;
    const size_t nvox = dims.width * dims.height * dims.depth;
    vr::SynthArgs a{};
    std::vector<float> gx, gy, gz;
    blob_tables(nx, ny, nz, seed, a, gx, gy, gz);
    std::vector<float> tab;
    if (nbins > 1) {
        tab.resize((size_t)vr::kSynthG * vr::kSynthQ * nbins);
        std::vector<double> e(nbins);
        for (int gi = 0; gi < vr::kSynthG; gi++) {
            const double sig = 0.02 + 0.1 * (double)gi / 15.0;
            for (int q = 0; q < vr::kSynthQ; q++) {
                const double mu = ((double)q + 0.5) / (double)vr::kSynthQ;
                double sum = 0.0;
                for (int b = 0; b < nbins; b++) {
                    const double dd = ((double)b + 0.5) / (double)nbins - mu;
                    e[b] = std::exp(-dd * dd / (2.0 * sig * sig));
                    sum += e[b];
                }
                float *row = tab.data() + ((size_t)gi * vr::kSynthQ + q) * nbins;
                for (int b = 0; b < nbins; b++) row[b] = (float)(e[b] / sum);
            }
        }
    }
    release_volume();
    uint64_t sy, sz;
    choose_pitch(nx, ny, sy, sz);
    float *vol = nullptr, *dgx = nullptr, *dgy = nullptr, *dgz = nullptr, *dtab = nullptr;
    auto cleanup = [&]() {
        if (dgx) (void)hipFree(dgx);
        if (dgy) (void)hipFree(dgy);
        if (dgz) (void)hipFree(dgz);
        if (dtab) (void)hipFree(dtab);
    };
    (void)nvox;
    hipError_t e = hipMalloc(&vol, sz * (size_t)nz * (size_t)nbins * sizeof(float));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(volume)");
    e = hipMalloc(&dgx, gx.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgy, gy.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgz, gz.size() * 4);
    if (e == hipSuccess && !tab.empty()) e = hipMalloc(&dtab, tab.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(dgx, gx.data(), gx.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgy, gy.data(), gy.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgz, gz.data(), gz.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && dtab)
        e = hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        a.gx = dgx; a.gy = dgy; a.gz = dgz; a.table = dtab;
        a.nx = nx; a.ny = ny; a.nz = nz; a.nb = nbins; a.seed = seed;
        a.sy = sy; a.sz = sz;
        e = vr::launch_synth(vol, a, g.stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    cleanup();
    if (e != hipSuccess) {
        (void)hipFree(vol);
        return hip_fail(e, "vr_synthesize");
    }
    g.vol = vol;
    g.owned = true;
    g.nx = nx; g.ny = ny; g.nz = nz; g.nb = nbins;
    g.sy = sy; g.sz = sz;
    return VR_OK;
}

int vr_set_layout_budget(uint64_t bytes) {
    g.layout_budget = bytes;
    // copies already resident beyond a lowered budget are dropped (the next
    // frame that wants one makes it again if it fits)
    if (layout_resident() > layout_budget_bytes()) {
        release_brick();
        release_axis_copy();
        release_plane_copies();
    }
    return VR_OK;
}

int vr_layout_info(uint64_t *resident_bytes, int *builds, float *last_build_ms,
                   uint64_t *last_build_bytes) {
    if (resident_bytes) *resident_bytes = layout_resident();
    if (builds) *builds = g.layout_builds;
    if (last_build_ms) *last_build_ms = g.layout_last_ms;
    if (last_build_bytes) *last_build_bytes = g.layout_last_bytes;
    return VR_OK;
}

int vr_volume_layout(size_t *row_pitch, size_t *slice_pitch) {
    if (!g.vol) return fail(VR_ERR_STATE, "no volume resident");
    if (row_pitch) *row_pitch = (size_t)g.sy;
    if (slice_pitch) *slice_pitch = (size_t)g.sz;
    return VR_OK;
}

int vr_volume_info(vr_extent *dims, int *nbins, const float **d_bins) {
    if (!g.vol) return fail(VR_ERR_STATE, "no volume resident");
    if (dims) {
        dims->width = (size_t)g.nx;
        dims->height = (size_t)g.ny;
        dims->depth = (size_t)g.nz;
    }
    if (nbins) *nbins = g.nb;
    if (d_bins) *d_bins = g.vol;
    return VR_OK;
}

}  // extern "C"

namespace {

// One frame of vr_render / render_kernel; clip_w x clip_h is the top-left
// rectangle of pixels the launch covers (render_kernel's gridSize x blockSize,
// K:2397 + K:282-286; the whole image otherwise).
int render_frame(const vr_render_desc *desc, uint32_t clip_w, uint32_t clip_h) {
    vr::Params P;
    uint32_t nslots = 0;
    int rc = fill_params(desc, P, nslots, true);
    if (rc != VR_OK) return rc;
    P.CW = std::min(clip_w, P.W);
    P.CH = std::min(clip_h, P.H);
    if (P.CW < P.W || P.CH < P.H) {
        // the launch keeps the whole frame's tiles and order; pixels outside
        // the rectangle leave at once (miss-free: nothing written), and the
        // frame records no tile costs for the adaptive order
        if (desc->d_tile_list) return fail(VR_ERR_ARG, "a clipped render takes the whole frame");
        if (P.CW == 0 || P.CH == 0) return VR_OK;
        P.tile_cost = nullptr;
    }
    // VR_DRY (tooling: tools/host_cost.py): the host work of a frame without its
    // launch, to time what a frame costs the issuing thread
    if (const char *e = vr::tuning("VR_DRY"))
        if (std::atoi(e) != 0) return VR_OK;
    hipError_t e;
    const int qm = desc->query_method;
    const float *baked = (qm >= 1 && qm <= 3 && g.stats)   ? g.stats + (uint64_t)(qm - 1) * g.stats_plane
                         : (qm >= 4 && qm <= 6 && g.cstats) ? g.cstats + (uint64_t)(qm - 4) * g.cstats_plane
                                                            : nullptr;
    if (qm == 7 && g.stats) {
        // method 7 from the baked corner means (plane 3): the same corner cache
        // and double lerps (K:395-480), 4 bytes per corner refresh
        P.nb = 1;
        P.sy = g.stats_sy;
        P.sz = g.stats_sz;
        e = vr::launch_march(1, -7, g.stats + 3 * g.stats_plane, P, nslots, false, g.stream);
    } else if (baked) {
        // one float per corner voxel, the same filter and composite (vr_stats.hip),
        // addressed in the planes' bricks
        P.nb = 1;
        P.sy = qm <= 3 ? g.stats_sy : g.cstats_sy;
        P.sz = qm <= 3 ? g.stats_sz : g.cstats_sz;
        // side / top views of the raw planes: the method's plane with the view's
        // axis in the brick rows (ensure_plane_copy), marched as row-aligned
        P.plane_axis = 0;
        if (qm <= 3 && std::fabs(desc->inv_view[0]) < 0.95f) {
            int ax = std::fabs(desc->inv_view[8]) >= 0.95f ? 2
                         : std::fabs(desc->inv_view[4]) >= 0.95f ? 1 : 0;
            // oblique views: the 8 x 2 x 2 brick copy (axis 3)
            if (!ax) ax = 3;
            if (ensure_plane_copy(qm - 1, ax)) {
                const State::PlaneCopy &c = g.pcopy[ax - 1][qm - 1];
                baked = c.buf;
                P.sy = c.sy;
                P.sz = c.sz;
                P.plane_axis = ax;
            }
        }
        P.path = baked_path(desc, P);
        // method 0: the 32-bit plane index (MODE 1), or a plane copy's MODE 4 / 5
        // (32-bit in-slice offsets, 64-bit slice offsets: ensure_plane_copy keeps
        // a slice < 2^32 floats, so a copy never needs -1, which reads x rows);
        // method -1: x-row planes too large for 32-bit indices (MODE 2).
        // VR_PLANE_WIDE=1 (tests) sends every x-row plane to -1.
        const char *ew = vr::tuning("VR_PLANE_WIDE");
        const bool wide = ew && std::atoi(ew) != 0;
        const bool narrow = P.plane_axis != 0 || (!wide && plane_narrow(P.sy, P.sz, (uint64_t)P.nz));
        e = vr::launch_march(1, narrow ? 0 : -1, baked, P, nslots, false, g.stream);
    } else if (is_flex_method(desc->query_method)) {
        e = vr::launch_march_flex(desc->query_method, P, nslots, g.stream);
    } else if (desc->query_method >= 4 && desc->query_method <= 6) {
        // the one-lane codec march of a row-aligned view: a 16x4 pixel block per
        // wave (1024^3 x 8 1080p C0 m4 2.91 -> 2.88 ms, m5 5.26 -> 5.17, m6 7.07 ->
        // 6.90; profiles/r06/segmap/codec_*.log); VR_CODEC_MAP=0/1 overrides
        P.seg_map = std::fabs(desc->inv_view[0]) >= 0.95f;
        if (const char *em = vr::tuning("VR_CODEC_MAP")) P.seg_map = std::atoi(em) != 0;
        e = vr::launch_march_codec(P.nb, desc->query_method, P, nslots, false, g.stream);
        if (e == hipErrorInvalidValue)
            return fail(VR_ERR_UNSUPPORTED, "codec volumes with %d bins (compiled: 1,2,4,8,16,32)",
                        P.nb);
    } else {
        // the quad marches of oblique views (methods 1/2/3 on path 0; method 7
        // when its grid is the volume's) read the micro-brick copy
        const char *eq = vr::tuning("VR_M7_QUAD");
        const bool m7_quad = qm == 7 && P.oblique && P.m7x == P.nx && P.m7y == P.ny &&
                             P.m7z == P.nz && !(eq && std::atoi(eq) == 0);
        // views whose screen x runs along the volume's z or y read that axis'
        // rows copy with the per-ray pipelined march (fill_params); if the copy
        // cannot be made (HBM), the oblique view's march on the x rows / bricks
        if (P.axis_view && !ensure_axis_copy(P.axis_view)) {
            P.axis_view = 0;
            P.path = 0;
        }
        if (P.axis_view) {
            const State::AxisCopy &c = g.acopy[P.axis_view - 1];
            P.avol = c.buf;
            P.asx = c.sx;
            P.asy = c.sy;
            P.asz = c.sz;
        } else if (g.nb == 8 && ((P.path == 0 && qm >= 1 && qm <= 3) || m7_quad) &&
                   ensure_brick()) {
            P.bvol = g.brick;
            P.bsy = g.bsy;
            P.bsz = g.bsz;
        }
        e = vr::launch_march(g.nb, desc->query_method, g.vol, P, nslots, false, g.stream);
    }
    if (e != hipSuccess) return hip_fail(e, "launch(k_march)");
    if (P.tile_cost) g.cost_recorded = true;
    return VR_OK;
}

}  // namespace

extern "C" {

int vr_render(const vr_render_desc *desc) { return render_frame(desc, UINT32_MAX, UINT32_MAX); }

int vr_debug_wave_clock(uint64_t *d_buf) {
    g.wave_clock = reinterpret_cast<unsigned long long *>(d_buf);
    return VR_OK;
}

// tooling: 6 x u64 device counters of the LDS-box marches (k_march /
// k_march_duo staged reads; layout in vr.h: [0] violations, [1] worst overrun,
// [2] out-of-volume box voxels, [3] decoded voxels, [4] lane slots, [5] spare),
// zeroed here on the library's stream and accumulated by every later launch;
// counted only by a -DVR_BOX_CHECK build, which reports whether it was built
// so (return 1) -- the default build returns 0
int vr_debug_box_check(uint64_t *d_buf) {
    if (d_buf) VR_HIP(hipMemsetAsync(d_buf, 0, 6 * sizeof(uint64_t), g.stream));
    g.box_check = reinterpret_cast<unsigned long long *>(d_buf);
#ifdef VR_BOX_CHECK
    return 1;
#else
    return 0;
#endif
}

int64_t vr_count_footprint(const vr_render_desc *desc) {
    vr::Params P;
    uint32_t nslots = 0;
    int rc = fill_params(desc, P, nslots);
    if (rc != VR_OK) return rc;
    if (desc->query_method < 1 || desc->query_method > 3)
        return fail(VR_ERR_UNSUPPORTED, "footprint count is defined for methods 1/2/3");
    const uint64_t nvox = (uint64_t)g.nx * g.ny * g.nz;
    const uint64_t nwords = (nvox + 63) / 64;
    unsigned long long *bits = nullptr, *total = nullptr;
    VR_HIP(hipMalloc(&bits, nwords * 8 + 8));
    total = bits + nwords;
    hipError_t e = hipMemsetAsync(bits, 0, nwords * 8 + 8, g.stream);
    P.mark = bits;
    if (e == hipSuccess)
        e = vr::launch_march(g.nb, desc->query_method, g.vol, P, nslots, true, g.stream);
    if (e == hipSuccess) e = vr::launch_popcount(bits, nwords, total, g.stream);
    unsigned long long u = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&u, total, 8, hipMemcpyDeviceToHost, g.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    (void)hipFree(bits);
    if (e != hipSuccess) return hip_fail(e, "vr_count_footprint");
    return (int64_t)u;
}

int64_t vr_footprint_bytes(const vr_render_desc *desc) {
    vr::Params P;
    uint32_t nslots = 0;
    int rc = fill_params(desc, P, nslots);
    if (rc != VR_OK) return rc;
    const int m = desc->query_method;
    if (m == 7 || m < 1 || m > 6)
        return fail(VR_ERR_UNSUPPORTED, "footprint bytes are defined for methods 1-6");
    if (m <= 3) {
        const int64_t u = vr_count_footprint(desc);
        return u < 0 ? u : u * (int64_t)g.nb * 4;
    }
    const uint64_t nvox = (uint64_t)P.nx * P.ny * P.nz;
    const uint64_t nwords = (nvox + 63) / 64;
    unsigned long long *bits = nullptr;
    VR_HIP(hipMalloc(&bits, nwords * 8 + 8));
    unsigned long long *total = bits + nwords;
    hipError_t e = hipMemsetAsync(bits, 0, nwords * 8 + 8, g.stream);
    P.mark = bits;
    if (e == hipSuccess) e = vr::launch_march_codec(P.nb, m, P, nslots, true, g.stream);
    if (e == hipSuccess) e = vr::launch_codec_bytes(bits, nvox, g.cb, total, g.stream);
    unsigned long long b = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&b, total, 8, hipMemcpyDeviceToHost, g.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    (void)hipFree(bits);
    if (e != hipSuccess) return hip_fail(e, "vr_footprint_bytes");
    return (int64_t)b + (int64_t)g.ntpl * g.cnb * 4;  // + the template table, read once
}

int vr_unscatter_tiles(const uint32_t *d_packed, const uint32_t *d_tile_lists, uint32_t n_ranks,
                       uint32_t n_slots, uint32_t *d_frame, uint32_t width, uint32_t height) {
    if (!d_packed || !d_tile_lists || !d_frame) return fail(VR_ERR_ARG, "null pointer");
    const uint64_t n = (uint64_t)n_ranks * n_slots;
    if (n > 0x7FFFFFFFull) return fail(VR_ERR_ARG, "too many tiles");
    hipError_t e = vr::launch_unscatter(d_packed, d_tile_lists, (uint32_t)n, tiles_x(width),
                                        d_frame, width, height, g.stream);
    if (e != hipSuccess) return hip_fail(e, "launch(k_unscatter)");
    return VR_OK;
}

// ---------------- GMM volumes (config 5) ----------

}  // extern "C"

namespace {

void release_gmm_volume(State::Gmm &v) {
    if (v.owned) {
        if (v.wm) (void)hipFree(v.wm);
        if (v.sg) (void)hipFree(v.sg);
    }
    v = State::Gmm{};
}

// the selected slot's GMM volume
void release_gmm() {
    g.volume_epoch++;
    release_gmm_volume(g.gmm);
}

// both slots' (freeCudaBuffers)
void release_all_gmm() {
    release_gmm();
    release_gmm_volume(g.gmm_parked[0]);
    release_gmm_volume(g.gmm_parked[1]);
    g.gmm_slot = 0;
}

int check_gmm_shape(vr_extent dims, int K, int z_base, int nzs) {
    if (K != 8 && K != 16 && K != 32)
        return fail(VR_ERR_UNSUPPORTED, "GMM volumes with %d components (compiled: 8, 16, 32)", K);
    if (dims.width == 0 || dims.height == 0 || dims.depth == 0 || dims.width > 65536 ||
        dims.height > 65536 || dims.depth > 65536)
        return fail(VR_ERR_ARG, "GMM volume: bad dims");
    // a slice must stay below 2^31 voxels: the march offsets corners by 32-bit slice strides
    if ((uint64_t)dims.width * dims.height >= (1ull << 31))
        return fail(VR_ERR_ARG, "GMM volume: a slice of %zu x %zu voxels is too large", dims.width,
                    dims.height);
    if (z_base < 0 || nzs < 1 || (size_t)z_base + (size_t)nzs > dims.depth)
        return fail(VR_ERR_ARG, "GMM volume: resident slices [%d, %d) outside [0, %zu)", z_base,
                    z_base + nzs, dims.depth);
    return VR_OK;
}

// Parameters of a GMM launch: the reference's ray / transfer / composite
// inputs from the descriptor, the resident slices, and the slab.
int fill_gmm_params(const vr_render_desc *d, const vr_gmm_slab *slab, vr::Params &P,
                    uint32_t &nblocks) {
    if (!d) return fail(VR_ERR_ARG, "null render descriptor");
    if (!g.gmm.wm) return fail(VR_ERR_STATE, "no GMM volume resident (vr_init_gmm / vr_synthesize_gmm)");
    if (d->query_method != 1 && d->query_method != 2)
        return fail(VR_ERR_UNSUPPORTED, "GMM volumes support queryMethod 1 (mean) and 2 (variance)");
    if (!d->d_output) return fail(VR_ERR_ARG, "d_output is null");
    if (d->width == 0 || d->height == 0) return fail(VR_ERR_ARG, "empty image");
    if ((uint64_t)d->width * d->height > 0xFFFFFFFFull) return fail(VR_ERR_ARG, "image too large");
    if (d->d_tile_list) return fail(VR_ERR_UNSUPPORTED, "GMM renders take whole frames or alive lists");
    std::memset(&P, 0, sizeof P);
    std::memcpy(P.m, d->inv_view, sizeof P.m);
    P.W = d->width;
    P.H = d->height;
    P.CW = d->width;
    P.CH = d->height;
    P.density = d->density;
    P.brightness = d->brightness;
    P.toff = d->transfer_offset;
    P.tscale = d->transfer_scale;
    P.nx = g.gmm.nx; P.ny = g.gmm.ny; P.nz = g.gmm.nz;
    P.gwm = g.gmm.wm;
    P.gsg = g.gmm.sg;
    P.gk = g.gmm.K;
    P.z_base = g.gmm.z_base;
    P.nzs = g.gmm.nzs;
    P.tiles_x = tiles_x(d->width);
    P.out = d->d_output;
    P.out_f = d->d_output_f;
    P.out_n = d->d_steps;
    device_lds(P.lds_cu, P.lds_wg);
    if (const char *e = vr::tuning("VR_WG_PER_CU")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= 32) P.wg_per_cu = v;
    }
    // lockstep batches (path 1, default): a wave's rays stay adjacent and at the
    // same step, so their corner loads share lines (1024^3 x 16, 1080p: C0
    // 4.89 -> 4.20 ms, C1 7.88 -> 7.38); VR_GMM_LOCKSTEP=0 refills groups one by one
    P.path = 1;
    if (const char *e = vr::tuning("VR_GMM_LOCKSTEP")) P.path = std::atoi(e) ? 1 : 0;
    const int zr_hi = g.gmm.z_base + g.gmm.nzs;  // resident slices end (exclusive)
    if (!slab) {
        if (g.gmm.z_base != 0 || g.gmm.nzs != g.gmm.nz)
            return fail(VR_ERR_STATE, "only slices [%d, %d) of the GMM volume are resident: "
                        "render it slab by slab (vr_render_gmm with a vr_gmm_slab)",
                        g.gmm.z_base, zr_hi);
        P.z_lo = 0;
        P.z_hi = g.gmm.nz;
    } else {
        if (slab->z_lo < 0 || slab->z_hi > g.gmm.nz || slab->z_lo >= slab->z_hi)
            return fail(VR_ERR_ARG, "slab [%d, %d) outside the volume's [0, %d)", slab->z_lo,
                        slab->z_hi, g.gmm.nz);
        // a footprint with z0 in [z_lo, z_hi) reads slices z0 and min(z0 + 1, nz - 1)
        const int need_hi = std::min(slab->z_hi + 1, g.gmm.nz);
        if (slab->z_lo < g.gmm.z_base || need_hi > zr_hi)
            return fail(VR_ERR_ARG, "slab [%d, %d) needs slices [%d, %d); resident: [%d, %d)",
                        slab->z_lo, slab->z_hi, slab->z_lo, need_hi, g.gmm.z_base, zr_hi);
        if (!slab->d_rays_out || !slab->d_n_rays_out)
            return fail(VR_ERR_ARG, "a slab launch needs d_rays_out and d_n_rays_out");
        if (slab->n_rays_in && !slab->d_rays_in) return fail(VR_ERR_ARG, "d_rays_in is null");
        if ((uint64_t)slab->n_rays_in > (uint64_t)d->width * d->height)
            return fail(VR_ERR_ARG, "%u alive rays in for a %ux%u frame", slab->n_rays_in,
                        d->width, d->height);
        // an alive-list entry holds the pixel in 23 bits (vr_gmm.hip GmmRay)
        if ((uint64_t)d->width * d->height > (1ull << 23))
            return fail(VR_ERR_ARG, "slab chains address at most 2^23 pixels (%ux%u)",
                        d->width, d->height);
        // slabs must be taken in the order every ray crosses them: the sign of
        // a ray's z step is that of the linear form u M8 + v M9 - 2 M10, so the
        // four frame corners decide whether it is the same for the whole frame
        const float *M = d->inv_view;
        int pos = 0, neg = 0;
        for (int c = 0; c < 4; c++) {
            const float u = (c & 1) ? ((float)(d->width - 1) / (float)d->width) * 2.0f - 1.0f : -1.0f;
            const float v = (c & 2) ? ((float)(d->height - 1) / (float)d->height) * 2.0f - 1.0f : -1.0f;
            const float dz = u * M[8] + v * M[9] - 2.0f * M[10];
            pos += dz > 0.0f;
            neg += dz < 0.0f;
        }
        if (pos && neg)
            return fail(VR_ERR_UNSUPPORTED, "rays of this view cross z-slabs in both directions: "
                        "slab-chained rendering needs one crossing order");
        P.z_lo = slab->z_lo;
        P.z_hi = slab->z_hi;
        P.rays_in = reinterpret_cast<const uint32_t *>(slab->d_rays_in);
        P.n_rays_in = slab->d_rays_in ? slab->n_rays_in : 0;
        P.rays_out = reinterpret_cast<uint32_t *>(slab->d_rays_out);
        P.n_rays_out = slab->d_n_rays_out;
    }
    if (P.rays_in || (slab && slab->d_rays_in)) {
        nblocks = (uint32_t)(((uint64_t)P.n_rays_in + 255) / 256);
        P.n_tiles = nblocks;
    } else {
        nblocks = tiles_x(d->width) * tiles_y(d->height);
        P.n_tiles = nblocks;
        int rc = frame_order(d, tiles_x(d->width), tiles_y(d->height), P.perm, nullptr);
        if (rc != VR_OK) return rc;
    }
    return VR_OK;
}

}  // namespace

extern "C" {

int vr_init_gmm(const float *wm, const float *sigma, vr_extent dims, int ncomp, int z_base,
                int nslices, int where) {
    int rc = check_gmm_shape(dims, ncomp, z_base, nslices);
    if (rc != VR_OK) return rc;
    if (!wm || !sigma) return fail(VR_ERR_ARG, "vr_init_gmm: null plane");
    if (where < 0 || where > 2) return fail(VR_ERR_ARG, "vr_init_gmm: where must be 0, 1 or 2");
    const uint64_t nvox = (uint64_t)dims.width * dims.height * (uint64_t)nslices;
    const size_t bwm = nvox * (size_t)ncomp * 8, bsg = nvox * (size_t)ncomp * 4;
    release_gmm();
    State::Gmm m;
    m.nx = (int)dims.width; m.ny = (int)dims.height; m.nz = (int)dims.depth;
    m.K = ncomp; m.z_base = z_base; m.nzs = nslices;
    if (where == 2) {
        m.wm = const_cast<float *>(wm);
        m.sg = const_cast<float *>(sigma);
        m.owned = false;
    } else {
        hipError_t e = hipMalloc(&m.wm, bwm);
        if (e == hipSuccess) e = hipMalloc(&m.sg, bsg);
        const hipMemcpyKind k = where == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
        if (e == hipSuccess) e = hipMemcpy(m.wm, wm, bwm, k);
        if (e == hipSuccess) e = hipMemcpy(m.sg, sigma, bsg, k);
        if (e != hipSuccess) {
            if (m.wm) (void)hipFree(m.wm);
            if (m.sg) (void)hipFree(m.sg);
            return hip_fail(e, "vr_init_gmm");
        }
        m.owned = true;
    }
    g.gmm = m;
    return VR_OK;
}

int vr_synthesize_gmm(vr_extent dims, int ncomp, uint64_t seed, int z_base, int nslices) {
    int rc = check_gmm_shape(dims, ncomp, z_base, nslices);
    if (rc != VR_OK) return rc;
    const int nx = (int)dims.width, ny = (int)dims.height, nz = (int)dims.depth;
    const uint64_t nvox = (uint64_t)nx * ny * (uint64_t)nslices;
    vr::SynthArgs a{};
    std::vector<float> gx, gy, gz;
    blob_tables(nx, ny, nz, seed, a, gx, gy, gz);
    release_gmm();
    State::Gmm m;
    float *dgx = nullptr, *dgy = nullptr, *dgz = nullptr;
    hipError_t e = hipMalloc(&m.wm, nvox * (size_t)ncomp * 8);
    if (e == hipSuccess) e = hipMalloc(&m.sg, nvox * (size_t)ncomp * 4);
    if (e == hipSuccess) e = hipMalloc(&dgx, gx.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgy, gy.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&dgz, gz.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(dgx, gx.data(), gx.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgy, gy.data(), gy.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgz, gz.data(), gz.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        a.gx = dgx; a.gy = dgy; a.gz = dgz;
        a.nx = nx; a.ny = ny; a.nz = nz; a.nb = ncomp; a.seed = seed;
        e = vr::launch_synth_gmm(m.wm, m.sg, a, ncomp, z_base, nslices, g.stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    if (dgx) (void)hipFree(dgx);
    if (dgy) (void)hipFree(dgy);
    if (dgz) (void)hipFree(dgz);
    if (e != hipSuccess) {
        if (m.wm) (void)hipFree(m.wm);
        if (m.sg) (void)hipFree(m.sg);
        return hip_fail(e, "vr_synthesize_gmm");
    }
    m.nx = nx; m.ny = ny; m.nz = nz; m.K = ncomp; m.z_base = z_base; m.nzs = nslices;
    m.owned = true;
    g.gmm = m;
    return VR_OK;
}

int vr_gmm_info(vr_extent *dims, int *ncomp, int *z_base, int *nslices, const float **d_wm,
                const float **d_sigma) {
    if (!g.gmm.wm) return fail(VR_ERR_STATE, "no GMM volume resident");
    if (dims) {
        dims->width = (size_t)g.gmm.nx;
        dims->height = (size_t)g.gmm.ny;
        dims->depth = (size_t)g.gmm.nz;
    }
    if (ncomp) *ncomp = g.gmm.K;
    if (z_base) *z_base = g.gmm.z_base;
    if (nslices) *nslices = g.gmm.nzs;
    if (d_wm) *d_wm = g.gmm.wm;
    if (d_sigma) *d_sigma = g.gmm.sg;
    return VR_OK;
}

int vr_gmm_select(int slot) {
    if (slot != 0 && slot != 1) return fail(VR_ERR_ARG, "GMM slot %d (0 or 1)", slot);
    if (slot == g.gmm_slot) return VR_OK;
    g.gmm_parked[g.gmm_slot] = g.gmm;
    g.gmm = g.gmm_parked[slot];
    g.gmm_parked[slot] = State::Gmm{};
    g.gmm_slot = slot;
    g.volume_epoch++;  // (the tile order is keyed on what is resident)
    return VR_OK;
}

int vr_free_gmm(void) {
    release_gmm();
    return VR_OK;
}

int vr_render_gmm(const vr_render_desc *desc, const vr_gmm_slab *slab) {
    vr::Params P;
    uint32_t nblocks = 0;
    int rc = fill_gmm_params(desc, slab, P, nblocks);
    if (rc != VR_OK) return rc;
    // the alive-list counter starts from 0 on the stream the launch runs on
    // (a caller zeroing it on another stream raced the launch)
    hipError_t e = slab ? hipMemsetAsync(slab->d_n_rays_out, 0, sizeof(uint32_t), g.stream)
                        : hipSuccess;
    if (e == hipSuccess)
        e = vr::launch_march_gmm(g.gmm.K, desc->query_method, P, nblocks, false, g.stream);
    if (e != hipSuccess) return hip_fail(e, "launch(k_march_gmm)");
    return VR_OK;
}

int64_t vr_gmm_count_footprint(const vr_render_desc *desc) {
    return vr_gmm_count_footprint_slab(desc, nullptr);
}

int64_t vr_gmm_count_footprint_slab(const vr_render_desc *desc, const vr_gmm_slab *slab) {
    vr::Params P;
    uint32_t nblocks = 0;
    int rc = fill_gmm_params(desc, slab, P, nblocks);
    if (rc != VR_OK) return rc;
    // one bit per resident voxel (gmm_vox indexes the resident slices)
    const uint64_t nvox = (uint64_t)g.gmm.nx * g.gmm.ny * (uint64_t)g.gmm.nzs;
    const uint64_t nwords = (nvox + 63) / 64;
    unsigned long long *bits = nullptr;
    VR_HIP(hipMalloc(&bits, nwords * 8 + 8));
    unsigned long long *total = bits + nwords;
    hipError_t e = hipMemsetAsync(bits, 0, nwords * 8 + 8, g.stream);
    if (e == hipSuccess && slab)
        e = hipMemsetAsync(slab->d_n_rays_out, 0, sizeof(uint32_t), g.stream);
    P.mark = bits;
    P.out = nullptr;  // count launch writes no pixels
    P.out_f = nullptr;
    P.out_n = nullptr;
    if (e == hipSuccess) e = vr::launch_march_gmm(g.gmm.K, desc->query_method, P, nblocks, true, g.stream);
    if (e == hipSuccess) e = vr::launch_popcount(bits, nwords, total, g.stream);
    unsigned long long u = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&u, total, 8, hipMemcpyDeviceToHost, g.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
    (void)hipFree(bits);
    if (e != hipSuccess) return hip_fail(e, "vr_gmm_count_footprint");
    return (int64_t)u;
}

// ---------------- reference entry points (K:1889-2406) ------------------

void render_kernel(vr_dim3 gridSize, vr_dim3 blockSize, uint32_t *d_output, uint32_t imageW,
                   uint32_t imageH, float density, float brightness, float transferOffset,
                   float transferScale, int queryMethod, vr_extent volumeSize) {
    // d_render covers x = blockIdx.x * blockDim.x + threadIdx.x < imageW (and
    // the same in y, K:282-286): a grid smaller than the image leaves the
    // pixels beyond gridSize x blockSize untouched, a larger one is cut at the
    // image.  A launch the reference's CUDA launch would refuse fails the same
    // way (cudaErrorInvalidConfiguration, reported by getLastCudaError, C:214):
    // an empty grid or block, more than 1024 threads per block, a block
    // dimension beyond (1024, 1024, 64) or a grid beyond (2^31 - 1, 65535, 65535).
    const uint64_t threads = (uint64_t)blockSize.x * blockSize.y * blockSize.z;
    if (gridSize.x == 0 || gridSize.y == 0 || gridSize.z == 0 || threads == 0 || threads > 1024 ||
        blockSize.x > 1024 || blockSize.y > 1024 || blockSize.z > 64 ||
        gridSize.x > 0x7FFFFFFFu || gridSize.y > 65535 || gridSize.z > 65535) {
        fail(VR_ERR_ARG, "render_kernel: invalid launch configuration grid (%u,%u,%u) block (%u,%u,%u)",
             gridSize.x, gridSize.y, gridSize.z, blockSize.x, blockSize.y, blockSize.z);
        return;
    }
    const uint64_t cw = (uint64_t)gridSize.x * blockSize.x, ch = (uint64_t)gridSize.y * blockSize.y;
    vr_render_desc d;
    std::memset(&d, 0, sizeof d);
    d.d_output = d_output;
    d.width = imageW;
    d.height = imageH;
    std::memcpy(d.inv_view, g.inv_view, sizeof d.inv_view);
    d.density = density;
    d.brightness = brightness;
    d.transfer_offset = transferOffset;
    d.transfer_scale = transferScale;
    d.query_method = queryMethod;
    d.volume_size = volumeSize;
    (void)render_frame(&d, (uint32_t)std::min<uint64_t>(cw, UINT32_MAX),
                       (uint32_t)std::min<uint64_t>(ch, UINT32_MAX));
}

void copyInvViewMatrix(float *invViewMatrix, size_t sizeofMatrix) {
    if (!invViewMatrix) {
        fail(VR_ERR_ARG, "copyInvViewMatrix: null matrix");
        return;
    }
    if (sizeofMatrix > sizeof g.inv_view) {
        fail(VR_ERR_ARG, "copyInvViewMatrix: %zu bytes > 48", sizeofMatrix);
        return;
    }
    std::memcpy(g.inv_view, invViewMatrix, sizeofMatrix);
}

void initCuda(void *h_histogram, vr_extent volumeSize, vr_extent histogramSize,
              vr_int4 *h_codebook, vr_extent codebookSize, float *h_templates,
              vr_extent templatesSize, vr_float2 *h_errorsbook, vr_extent errorsbookSize,
              vr_int4 *h_codebookSpanLow, vr_int4 *h_codebookSpanHigh,
              vr_int4 *h_flexibleCodebook, vr_float2 *h_flexibleErrorsbook,
              vr_int4 *h_simpleLow, vr_int4 *h_simpleHigh, int *h_simpleCount,
              vr_float2 *h_simpleHistogram, float *h_flexibleTemplates) {
    const size_t nvox = volumeSize.width * volumeSize.height * volumeSize.depth;
    if (histogramSize.width == 0 || histogramSize.height * histogramSize.depth != nvox) {
        fail(VR_ERR_ARG,
             "initCuda: histogramSize (%zu,%zu,%zu) does not hold one record per voxel of "
             "(%zu,%zu,%zu)",
             histogramSize.width, histogramSize.height, histogramSize.depth, volumeSize.width,
             volumeSize.height, volumeSize.depth);
        return;
    }
    if (vr_init_distribution((const float *)h_histogram, volumeSize, (int)histogramSize.width,
                             0) != VR_OK)
        return;
    g.linear_filter = false;
    // codec arrays (methods 4/5/6, K:1920-2050): codebook (X,Y,Z) int4, templates
    // (nBins, nTemplates, layers) -- layer 0 is used, the reference reads layer 1
    // of a 1-layer array (K:792-793) --, errorsbook (slots, rows, layers) with one
    // row of `slots` (bin, error) pairs per voxel
    if (h_codebook && h_templates && h_errorsbook) {
        if (codebookSize.width != volumeSize.width || codebookSize.height != volumeSize.height ||
            codebookSize.depth != volumeSize.depth || templatesSize.width != histogramSize.width ||
            errorsbookSize.height * errorsbookSize.depth != nvox) {
            fail(VR_ERR_ARG, "initCuda: codebook/templates/errorsbook sizes do not match the volume");
            return;
        }
        (void)vr_init_codec(h_codebook, codebookSize, h_templates, (int)templatesSize.height,
                            h_errorsbook, (int)errorsbookSize.width, (int)templatesSize.width, 0);
    }
    // flexible-block span tables (methods 8/9/0, K:2052-2320) with the
    // reference's fixed sizes: 64x64x32 fractal and simple entries
    // (flexibleVolumeSize, K:99), 64 bins, 469 templates (K:98, 101), a 64^3
    // raw volume (K:106)
    if (h_codebookSpanLow && h_codebookSpanHigh && h_flexibleCodebook && h_flexibleErrorsbook &&
        h_simpleLow && h_simpleHigh && h_simpleCount && h_simpleHistogram && h_flexibleTemplates) {
        vr_flex_tables t;
        t.dim = 64;
        t.nbins = 64;
        t.n_fractal = t.n_simple = 64 * 64 * 32;
        t.fractal_low = h_codebookSpanLow;
        t.fractal_high = h_codebookSpanHigh;
        t.fractal_code = h_flexibleCodebook;
        t.fractal_errors = h_flexibleErrorsbook;
        t.simple_low = h_simpleLow;
        t.simple_high = h_simpleHigh;
        t.simple_count = h_simpleCount;
        t.simple_hist = h_simpleHistogram;
        t.templates = h_flexibleTemplates;
        t.ntemplates = 469;
        (void)vr_init_flex(&t);
    }
}

void freeCudaBuffers(void) {
    release_volume();
    release_codec();
    release_flex();
    release_all_gmm();
}

void setTextureFilterMode(bool bLinearFilter) { g.linear_filter = bLinearFilter; }

void basicDataProcessing(void) {
    // d_basicDataProcessing (K:1798-1887) fills originalQueryTex / fractalQueryTex
    // once; here the planes of vr_stats.hip.  Errors go to vr_last_error(); a
    // failed bake leaves the per-step decode in place.
    (void)bake_stats();
}

int vr_bake_stats(void) { return bake_stats(); }

int vr_release_stats(void) {
    release_stats();
    release_cstats();
    release_brick();  // the layout copies are derived from the records too
    release_axis_copy();
    return VR_OK;
}

int vr_stats_info(const float **d_raw, uint64_t *raw_plane, const float **d_codec,
                  uint64_t *codec_plane) {
    if (d_raw) *d_raw = g.stats;
    if (raw_plane) *raw_plane = g.stats_plane;
    if (d_codec) *d_codec = g.cstats;
    if (codec_plane) *codec_plane = g.cstats_plane;
    return VR_OK;
}

void dataProcessing(void) {
    (void)vr_flex_process(6);  // blockSize = 6, K:1737
}

}  // extern "C"

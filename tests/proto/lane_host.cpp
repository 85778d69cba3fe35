// TEST ONLY: host build of the lane kernels' per-lane compress/decompress
// (rc_lane3.hip) and, with -DDEC6, the fast decoder in front of them.
#define RC_LANE_HOST_TEST 1
#include <stdlib.h>
#include <string.h>
#include "../../enet_amd/csrc/rc_lane3.hip"
#ifdef DEC6
#include "../../enet_amd/csrc/rc_dec6.hip"
static uint8_t g_lds6[528] __attribute__((aligned(16)));   // root + bucket bytes
static uint8_t g_itab6[512] __attribute__((aligned(16)));  // root3_inc_init's table
static const uint8_t* itab6()
{
    static bool init = false;
    if (!init) { for (uint32_t g = 0; g < 16; ++g) root3_inc_init(g_itab6, g); init = true; }
    return g_itab6;
}
// -DDEC6S: the lane's input through the LDS slot (rc_slot.h), the helper's
// pass run after every step and whenever the lane waits
static uint32_t g_ctl6s[3];
static SlotHelp g_sh6;
static const rc_batch_dev* g_b6s = nullptr;
static uint32_t g_hcks6[2], g_icks6[1];           // the hand-off's check sums (rc_slot.h slot_mix)
namespace {
static void slot_host_kick()
{
    bool fin = false;
    if (g_b6s) slot_help_iter(*g_b6s, g_ctl6s, g_ctl6s + 2, g_lds6 + 256, g_sh6, g_hcks6, 1, fin);
}
static void slot_host_step() { slot_host_kick(); }
static void slot_host_point(int) {}                         // (interleavings: tests/proto/slot_sched.cpp)
// stale-chunk injection (tests/test_lane_host.py): the k-th chunk the lane
// takes from its slot replaced by kind 0: the chunk the slot held before it
// (the one the lane is on), 1: the chunk after it, 2: zeros
static int g_inj_take = -1, g_inj_kind = 0, g_inj_seen = 0;
static uintptr_t g_inj_lo = 0, g_inj_hi = 0;
static void slot_host_taken(uint32_t j, uint4& sl)
{
    if (g_inj_seen++ != g_inj_take) return;
    const uintptr_t base = g_inj_lo & ~static_cast<uintptr_t>(15);
    if (g_inj_kind == 0) sl = chunk_load(g_inj_lo, g_inj_hi, base + 16 * static_cast<uintptr_t>(j), true);
    else if (g_inj_kind == 1) sl = chunk_load(g_inj_lo, g_inj_hi, base + 16 * static_cast<uintptr_t>(j + 2), true);
    else sl = make_uint4(0u, 0u, 0u, 0u);
}
}  // namespace
static uint8_t g_tab6[RC_DEC6_TAB_BYTES] __attribute__((aligned(16)));   // bucket records (never cleared)

// rc_dec6_verify on the host: distinct bigrams of the output, per model
// segment (rst: the segments' starts after the first, as rc_dec6.hip records them)
static uint32_t distinct_bigrams(const uint8_t* x, uint32_t n, uint32_t rst = 0)
{
    static uint8_t seen[65536];
    uint32_t c = 0;
    const uint32_t nseg = (rst >> 24) + 1;
    for (uint32_t sg = 0; sg < nseg; ++sg) {
        const uint32_t s0 = sg ? (rst >> (12 * (sg - 1))) & 0xFFFu : 0u;
        const uint32_t s1 = sg + 1 < nseg ? (rst >> (12 * sg)) & 0xFFFu : n;
        memset(seen, 0, sizeof seen);
        for (uint32_t j = s0 + 1; j < s1; ++j) {
            const uint32_t b = (x[j - 1] << 8) | x[j];
            c += seen[b] ? 0u : 1u;
            seen[b] = 1;
        }
    }
    return c;
}
#endif

#define REGION_BYTES rc_hip_lane3_region_bytes
#define COMPRESS_ONE compress_one3
#define DECOMPRESS_ONE decompress_one3

static uint8_t g_root[304] __attribute__((aligned(16)));
static uint8_t g_mtab[256] __attribute__((aligned(16)));
static uint8_t g_ldsb[kDenseO2] __attribute__((aligned(16)));   // the lane's LDS dense block
static uint16_t g_lc[kLinkCache] __attribute__((aligned(16)));   // the decoder's link cache
static bool g_mtab_init = [] { for (uint32_t j = 0; j < 16; ++j) root3_mask_init(g_mtab, j); return true; }();
#define COMPRESS_ARGS , g_ldsb, g_mtab

static uint32_t g_dec6_unverified = 0;
extern "C" uint32_t lane_host_dec6_unverified(void) { return g_dec6_unverified; }
#ifdef DEC6S
// the next decode's take-th slot chunk replaced (kind: see slot_host_taken);
// returns the slot takes of the last decode
extern "C" int lane_host_inject(int take, int kind)
{
    const int seen = g_inj_seen;
    g_inj_take = take; g_inj_kind = kind;
    return seen;
}
#endif

extern "C" int lane_host_run(int decompress, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t cap,
                             uint32_t max_len, uint32_t* out_len)
{
    static uint8_t* region = nullptr;
    static uint32_t region_bytes = 0;
    uint32_t need = REGION_BYTES(max_len);
    if (need > region_bytes) {
        free(region); region = (uint8_t*) aligned_alloc(256, need); region_bytes = need;
        memset(region, 0, need);                                   // like the device pool (epoch 0 = unused)
    }
    uint64_t ioff = 0, ooff = 0;
    uint32_t flags[2] = {0, 0}, counters[4] = {0, 0, 0, 0}, bails[2] = {0, 0}, claims[1] = {0}, resets[1] = {0};
    rc_batch_dev b = { in, &ioff, &len, out, &ooff, &cap, out_len, 1, max_len };
    rc_workspace_dev ws = {};
    ws.flag_list = flags; ws.counters = counters; ws.enc2_list = bails; ws.lane_region = need; ws.lane_pool = region; ws.lane_active = 64;
    ws.claims = claims;
    ws.dec6_resets = resets;
    *out_len = 0xFFFFFFFFu;
#ifdef DEC6
    // the record-light decoder and its check; a packet it leaves or that fails the check goes to the lanes
    if (decompress) {
#ifndef DEC6S
        ByteSrc src6;
        decompress_one6(b, ws, 0, g_lds6, g_lds6 + kStats6, g_tab6, g_tab6 + kTab1, itab6(), src6);
        const bool ck = true;
#else
        g_b6s = &b;
        g_inj_seen = 0;
        g_inj_lo = reinterpret_cast<uintptr_t>(in); g_inj_hi = g_inj_lo + len;
        g_ctl6s[0] = 0u; g_ctl6s[1] = kNoPktS; g_ctl6s[2] = 0u;
        slot_help_init(g_sh6);
        SlotSrc src6;
        src6.gen = 0; src6.mctl = g_ctl6s; src6.hctl = g_ctl6s + 2; src6.slot = g_lds6 + 256;
        ws.dec6_icks = g_icks6; ws.dec6_hcks = g_hcks6;
        g_icks6[0] = 0; g_hcks6[0] = 0; g_hcks6[1] = 0;
        decompress_one6(b, ws, 0, g_lds6, g_lds6 + kStats6, g_tab6, g_tab6 + kTab1, itab6(), src6);
        g_ctl6s[1] = kFinS;                        // the lane is done: the helper stores its sum
        slot_host_kick();
        g_b6s = nullptr;
        const bool ck = cks_agree(g_icks6[0], g_hcks6[0], g_hcks6[1]);
#endif
        if (!counters[3] && (!ck || (claims[0] & 0x7FFFFFFFu) != distinct_bigrams(out, *out_len, resets[0]))) {
            counters[3] = 1; g_dec6_unverified++;
        }
        if (!counters[3] && (claims[0] >> 31)) *out_len = 0;
        if (!counters[3]) return 0;
    }
#endif

    if (decompress) DECOMPRESS_ONE(b, ws, 0, region, g_root, g_ldsb, g_lc);
    else COMPRESS_ONE(b, ws, 0, region, g_root COMPRESS_ARGS);
    return counters[0] ? 1 : (counters[3] ? 2 : 0);   // 1 = routed to the exact path, 2 = left by the fast decoder
}

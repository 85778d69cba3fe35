// TEST ONLY: the record-light decoder's input hand-off (enet_amd/csrc/rc_slot.h)
// under a seeded scheduler.  One decoding lane runs rc_dec6.hip's
// decompress_one6 over a run of packets (as a GPU lane does: one SlotSrc, its
// generation counting up, the LDS control words kept across packets) and its
// helper lane runs slot_help_iter, each on a thread of its own, exactly one of
// them running at a time.  At every point between two LDS word accesses of the
// protocol (SLOT_POINT in rc_slot.h: the decoder's h_ctl read, each dword of
// its slot read, its m_pkt and m_ctl stores; the helper's m_ctl and m_pkt
// reads, each dword of its slot store, its h_ctl store) the running side hands
// the turn to the other with probability p, drawn from a seeded generator, and
// a side that waits for the other (the decoder spinning on its slot, an idle
// helper) always hands it over.  Every chunk the decoder takes from the slot
// is checked against the packet's bytes (SLOT_TAKEN), and the decoded packets
// are returned for comparison with the oracle (tests/test_slot_sched.py).
//
// The model is weaker than gfx950's LDS (which performs one instruction
// whole, a wavefront's instructions in issue order): here every dword access
// is its own step.  SLOT_MUTANT=1 (the generation stored before the packet
// index: what a torn 64-bit store could show) and SLOT_MUTANT=2 (the helper's
// announcement before its slot store) are protocol faults the test must find.
#define RC_LANE_HOST_TEST 1
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <thread>

#include "../../enet_amd/csrc/rc_dec6.hip"

namespace {

std::mutex g_mu;
std::condition_variable g_cv;
int g_turn = 0;                       // 0: the decoding lane, 1: the helper
thread_local int t_me = -1;
uint64_t g_rng = 1;
uint32_t g_p16 = 0;                   // switch probability x 65536
uint64_t g_switches = 0;
bool g_done[2] = {false, false};      // a side that has finished takes no more turns
thread_local int32_t t_run = -1;      // bursts: points left in this turn (-1: draw at the next point)

uint32_t next_rand()
{
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return static_cast<uint32_t>((z ^ (z >> 31)) >> 16) & 0xFFFFu;
}

void handover()
{
    std::unique_lock<std::mutex> lk(g_mu);
    if (g_done[1 - t_me]) return;
    g_turn = 1 - t_me;
    ++g_switches;
    g_cv.notify_all();
    g_cv.wait(lk, [] { return g_turn == t_me || g_done[1 - t_me]; });
    t_run = -1;                       // (bursts: a new run drawn at the next point)
}

void finish()
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_done[t_me] = true;
    g_turn = 1 - t_me;
    g_cv.notify_all();
    t_me = -1;
}

void wait_turn()
{
    std::unique_lock<std::mutex> lk(g_mu);
    g_cv.wait(lk, [] { return g_turn == t_me; });
}

// the packet the decoding lane is on (for SLOT_TAKEN)
uintptr_t g_lo = 0, g_hi = 0;
uint32_t g_bad_takes = 0, g_takes = 0;

}  // namespace

namespace {
// p16 = 0: bursts instead -- each turn lasts a run of points drawn
// log-uniformly from 1..4096, so that long stretches of one side (a decoder
// consuming a whole chunk between two helper passes) are as likely as
// fine-grained alternation
static void new_run()
{
    t_run = 1 << (next_rand() % 13);
    t_run += static_cast<int32_t>(next_rand()) % t_run;
}
// p16 = 0xFFFF: per site -- every point (its source line) gets a switch
// probability of its own, drawn per run from {0, 1/256, 1/16, 1/2, 1}, so
// that a run can always switch at one point and never at another (a switch
// exactly between two stores, then a long stretch of the other side)
uint32_t g_site_p16[64];
static void draw_sites()
{
    static const uint32_t ps[5] = {0u, 256u, 4096u, 32768u, 65536u};
    for (uint32_t k = 0; k < 64; ++k) g_site_p16[k] = ps[next_rand() % 5];
}
// p16 = 0xFFFE: one site -- the sides run cooperatively (a side hands over
// only when it waits for the other) but for one point, chosen per run among
// the points met so far, which switches with probability 1/8, 1/2 or 1: a
// preemption at exactly one place, then each side for as long as it can go
int g_seen[64];
uint32_t g_nseen = 0;
int g_one_site = -1;
uint32_t g_one_p16 = 0;
static void draw_one_site()
{
    static const uint32_t ps[3] = {8192u, 32768u, 65536u};
    g_one_site = g_nseen ? g_seen[next_rand() % g_nseen] : -1;
    g_one_p16 = ps[next_rand() % 3];
}
static bool switch_now(int site)
{
    if (g_nseen < 64) {
        bool known = false;
        for (uint32_t k = 0; k < g_nseen; ++k) known = known || g_seen[k] == site;
        if (!known) g_seen[g_nseen++] = site;
    }
    if (g_p16 == 0xFFFEu) return site == g_one_site && next_rand() < g_one_p16;
    if (g_p16 == 0xFFFFu) return next_rand() < g_site_p16[static_cast<uint32_t>(site) % 61u];
    if (g_p16) return next_rand() < g_p16;
    if (t_run < 0) new_run();
    return --t_run <= 0;
}
static void slot_host_point(int site)
{
    if (t_me >= 0 && switch_now(site)) handover();
}
static void slot_host_kick()
{
    if (t_me == 0) handover();          // the decoding side waits for its helper
}
static void slot_host_step() { slot_host_point(__LINE__); }
static void slot_host_taken(uint32_t j, uint4& sl)
{
    const uint4 w = chunk_load(g_lo, g_hi, (g_lo & ~static_cast<uintptr_t>(15)) + 16 * static_cast<uintptr_t>(j + 1),
                               true);
    ++g_takes;
    if (w.x != sl.x || w.y != sl.y || w.z != sl.z || w.w != sl.w) ++g_bad_takes;
}
}  // namespace

static uint8_t g_lds[528 + 16] __attribute__((aligned(16)));
static uint8_t g_itab[512] __attribute__((aligned(16)));
static uint32_t g_ctl[3];
static uint8_t g_tab[RC_DEC6_TAB_BYTES] __attribute__((aligned(16)));

// Decodes packets 0..n-1 of the batch on one lane with its helper, under
// the scheduler seeded with `seed` (switch probability p16 / 65536 at each
// point; 0: bursts, 0xFFFF: per-site probabilities, 0xFFFE: one site).  out_len / claims /
// icks / hcks (the hand-off's check sums, rc_slot.h slot_mix; hcks[n + i]: the helper's last
// chunk's term): per packet (claims 0xFFFFFFFF:
// the packet left the fast decoder).  Returns the number of chunks taken that differ from the
// packet's bytes; *takes: chunks taken; *switches: hand-overs.
extern "C" uint32_t slot_sched_run(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                   uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                                   uint32_t* claims, uint32_t* icks, uint32_t* hcks, uint64_t seed, uint32_t p16,
                                   uint32_t* takes, uint64_t* switches)
{
    static bool init = false;
    if (!init) { for (uint32_t g = 0; g < 16; ++g) root3_inc_init(g_itab, g); init = true; }
    uint32_t counters[4] = {0, 0, 0, 0};
    uint32_t* bails = static_cast<uint32_t*>(calloc(n + 1, sizeof(uint32_t)));
    uint32_t* resets = static_cast<uint32_t*>(calloc(n + 1, sizeof(uint32_t)));
    rc_batch_dev b = {in, in_off, in_len, out, out_off, out_cap, out_len, n, 4096};
    rc_workspace_dev ws = {};
    ws.counters = counters; ws.enc2_list = bails; ws.lane_active = 64;
    ws.claims = claims;
    ws.dec6_resets = resets;
    ws.dec6_icks = icks;
    ws.dec6_hcks = hcks;
    g_rng = seed;
    g_p16 = p16;
    g_switches = 0;
    g_bad_takes = 0;
    g_takes = 0;
    g_turn = 0;
    g_done[0] = g_done[1] = false;
    draw_sites();
    draw_one_site();
    // the kernel's start (rc_decompress_dec6s): m_ctl / m_pkt before the first
    // packet, h_ctl 0
    g_ctl[0] = 0u; g_ctl[1] = n ? kNoPktS : kFinS; g_ctl[2] = 0u;
    uint8_t* slotp = g_lds + 256;
    memset(slotp, 0xA5, 16);

    std::thread helper([&] {
        t_me = 1;
        wait_turn();
        SlotHelp h;
        slot_help_init(h);
        for (;;) {
            bool fin = false;
            const bool busy = slot_help_iter(b, g_ctl, g_ctl + 2, slotp, h, hcks, n, fin);
            if (fin) break;
            if (!busy) handover();          // idle: the decoding side runs
            else slot_host_point(__LINE__);
        }
        finish();
    });

    t_me = 0;
    SlotSrc src;
    src.gen = 0; src.mctl = g_ctl; src.hctl = g_ctl + 2; src.slot = slotp;
    for (uint32_t pkt = 0; pkt < n; ++pkt) {
        g_lo = reinterpret_cast<uintptr_t>(in + in_off[pkt]);
        g_hi = g_lo + in_len[pkt];
        out_len[pkt] = 0xFFFFFFFFu;
        decompress_one6(b, ws, pkt, g_lds, g_lds + kStats6, g_tab, g_tab + kTab1, g_itab, src);
    }
    g_ctl[1] = kFinS;                      // the lane is done (rc_decompress_dec6s)
    finish();
    helper.join();
    free(bails);
    free(resets);
    *takes = g_takes;
    *switches = g_switches;
    return g_bad_takes;
}

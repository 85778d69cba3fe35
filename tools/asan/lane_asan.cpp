// Diagnostic (host only): the lane kernels' per-lane logic (tests/proto/lane_host.cpp)
// under AddressSanitizer, each packet in buffers of exactly its size, over a
// batch written by tools/asan_lane.py.  usage: lane_asan DIR
// Each buffer covers its packet's aligned 16-B granules (the kernels read and
// write whole aligned granules, which never cross a page, so they may touch
// the bytes around a packet in its first and last granule) with the packet at
// the alignment phase it has in the batch (phases.bin: input, output phase).
#include "../../tests/proto/lane_host.cpp"
#include <stdio.h>
#include <vector>

static std::vector<uint8_t> slurp(const char* dir, const char* name)
{
    char p[1024];
    snprintf(p, sizeof p, "%s/%s", dir, name);
    FILE* f = fopen(p, "rb");
    if (!f) { perror(p); exit(2); }
    std::vector<uint8_t> v;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
    fclose(f);
    return v;
}

// the aligned granules around len bytes at phase ph (0-15)
static uint8_t* granules(uint32_t ph, uint32_t len)
{
    const size_t bytes = (ph + len + 15) & ~static_cast<size_t>(15);
    return static_cast<uint8_t*>(aligned_alloc(16, bytes ? bytes : 16));
}

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    const auto d = slurp(argv[1], "data.bin"), c = slurp(argv[1], "comp.bin");
    const auto dlv = slurp(argv[1], "dlen.bin"), clv = slurp(argv[1], "clen.bin");
    const uint32_t* dl = reinterpret_cast<const uint32_t*>(dlv.data());
    const uint32_t* cl = reinterpret_cast<const uint32_t*>(clv.data());
    const auto phv = slurp(argv[1], "phases.bin");       // per packet: data phase, compressed phase
    const uint8_t* ph = phv.data();
    const size_t n = dlv.size() / 4;
    uint32_t dmax = 0, cmax = 0;
    for (size_t i = 0; i < n; ++i) { dmax = dl[i] > dmax ? dl[i] : dmax; cmax = cl[i] > cmax ? cl[i] : cmax; }
    size_t di = 0, ci = 0, bad = 0, exact = 0, left = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t ol = 0;
        // compress: cap 2 len + 64 (tools/soak.py)
        if (dl[i]) {
            uint8_t* ib = granules(ph[2 * i], dl[i]);
            uint8_t* in = ib + ph[2 * i];
            memcpy(in, d.data() + di, dl[i]);
            const uint32_t cap = 2 * dl[i] + 64;
            uint8_t* ob = granules(ph[2 * i + 1], cap);
            uint8_t* out = ob + ph[2 * i + 1];
            const int rc = lane_host_run(0, in, dl[i], out, cap, dmax, &ol);
            if (rc == 1) ++exact;
            else if (ol != cl[i] || memcmp(out, c.data() + ci, ol)) ++bad;
            free(ib); free(ob);
        }
        // decompress: cap = the packet's length, max_len = the largest compressed length (as the soak's calls)
        if (cl[i]) {
            uint8_t* ib = granules(ph[2 * i + 1], cl[i]);
            uint8_t* in = ib + ph[2 * i + 1];
            memcpy(in, c.data() + ci, cl[i]);
            uint8_t* ob = granules(ph[2 * i], dl[i]);
            uint8_t* out = ob + ph[2 * i];
            const int rc = lane_host_run(1, in, cl[i], out, dl[i], cmax, &ol);
            if (rc == 1) ++exact;
            else if (ol != dl[i] || memcmp(out, d.data() + di, ol)) ++bad;
            left += rc == 2;
            free(ib); free(ob);
        }
        di += dl[i]; ci += cl[i];
    }
    printf("packets %zu mismatches %zu exact %zu left %zu\n", n, bad, exact, left);
    return bad ? 1 : 0;
}

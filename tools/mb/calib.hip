// Calibration of the memory-side request counters (diagnostic, not product;
// round-5 review item 9): how the TCC_EA0 read / write request counters that
// tools/traffic.py turns into bytes tally the decoders' own access widths.
// Each kernel makes a known number of accesses of one width at random
// addresses over a table (as the decoders do: 65536 lanes, one access per
// lane and step), so requests per access and request sizes can be read off
// the counters of its own dispatch (rocprofv3 --pmc, tools/calib.sh):
//   st2   2-B store into a random 16-B record         (rc_dec6 element store)
//   st4   4-B store into a random 16-B record
//   st16  16-B store of a whole random 16-B record
//   ld16  16-B load of a random 16-B record           (rc_dec6 first record)
//   ld48  48-B load (3 x 16 B) of a random 48-B record (rc_dec6 second record)
//   ld64  64-B load (4 x 16 B) of a random 64-B record (rc_lane3 records)
//   seqst 16-B per lane coalesced streaming store     (reference: WRITE_SIZE exact)
//   seqld 16-B per lane coalesced streaming load      (reference: FETCH_SIZE = half)
// Tables: 1 GB (past the 256-MB Infinity Cache) and 64 MB (resident).
// Prints, per kernel, accesses and bytes the kernel moves by construction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kLanes = 65536, kSteps = 64;

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void calib(uint8_t* t, uint64_t recs, uint32_t* sink)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    const uint32_t rec = MODE == 4 ? 48 : MODE == 5 ? 64 : 16;
    for (uint32_t i = 0; i < kSteps; ++i) {
        const uint64_t r = (static_cast<uint64_t>(mix(lane * kSteps + i)) * recs) >> 32;
        uint8_t* p = t + r * rec;
        if (MODE == 0) *reinterpret_cast<uint16_t*>(p + 2 * (i & 7)) = static_cast<uint16_t>(lane + i);
        if (MODE == 1) *reinterpret_cast<uint32_t*>(p + 4 * (i & 3)) = lane + i;
        if (MODE == 2) *reinterpret_cast<uint4*>(p) = make_uint4(lane, i, lane + i, 1u);
        if (MODE >= 3 && MODE <= 5) {
            const uint4* q = reinterpret_cast<const uint4*>(p);
            const uint32_t k = rec / 16;
            for (uint32_t j = 0; j < k; ++j) { const uint4 w = q[j]; acc += w.x ^ w.w; }
        }
        if (MODE == 6) {
            uint4* q = reinterpret_cast<uint4*>(t) + (static_cast<uint64_t>(i) * kLanes + lane) % (recs);
            *q = make_uint4(lane, i, 0u, 1u);
        }
        if (MODE == 7) {
            const uint4* q = reinterpret_cast<const uint4*>(t) + (static_cast<uint64_t>(i) * kLanes + lane) % (recs);
            const uint4 w = *q;
            acc += w.y;
        }
    }
    if (acc == 0x12345678u) sink[lane] = acc;
}

template <int MODE>
void run(const char* name, uint8_t* t, uint64_t bytes, uint32_t* sink)
{
    const uint32_t rec = MODE == 4 ? 48 : MODE == 5 ? 64 : 16;
    const uint64_t recs = bytes / rec;
    hipLaunchKernelGGL(calib<MODE>, dim3(kLanes / 256), dim3(256), 0, 0, t, recs, sink);
    hipDeviceSynchronize();
    const uint64_t acc = static_cast<uint64_t>(kLanes) * kSteps;
    const uint32_t width = MODE == 0 ? 2 : MODE == 1 ? 4 : MODE == 4 ? 48 : MODE == 5 ? 64 : 16;
    printf("%-6s table %5llu MB  accesses %llu  width %u B  bytes %llu\n", name,
           static_cast<unsigned long long>(bytes >> 20), static_cast<unsigned long long>(acc), width,
           static_cast<unsigned long long>(acc * width));
}

int main()
{
    uint8_t* t = nullptr;
    uint32_t* sink = nullptr;
    const uint64_t big = 1ull << 30, small = 64ull << 20;
    if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&sink, kLanes * 4) != hipSuccess) return 1;
    hipMemset(t, 0, big);
    hipDeviceSynchronize();
    for (uint64_t bytes : {big, small}) {
        run<0>("st2", t, bytes, sink);
        run<1>("st4", t, bytes, sink);
        run<2>("st16", t, bytes, sink);
        run<3>("ld16", t, bytes, sink);
        run<4>("ld48", t, bytes, sink);
        run<5>("ld64", t, bytes, sink);
        run<6>("seqst", t, bytes, sink);
        run<7>("seqld", t, bytes, sink);
    }
    hipFree(t);
    hipFree(sink);
    return 0;
}

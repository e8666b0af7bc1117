// Device-side ingest of the example's input file data/matrix.in
// (examples/svd_example.rs:326-330, serde_json's default float path), for text
// already in device memory: a chunked three-pass scan over the bytes (string /
// bracket state, then counts, then positions and parsed numbers), after which
// the host resolves the few top-level keys and the arrays' number ranges.
// Same results as the host parser (csrc/ingest.hpp, kParseSerde) on every input
// it accepts; malformed inputs are rejected (SVDW_EINVAL).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svdw_ingest_dev {

static constexpr uint32_t kChunk = 4096;   // bytes per block (256 threads x 16)
// 2-state transfer of a byte range: f = the string state after the range for
// entry state 0 (outside) / 1 (inside a string) as bits 0 / 1; d0 / d1 = the
// bracket depth change for each entry state.
struct Xfer {
    int32_t f, d0, d1;
};
// per chunk: numbers, row opens ('[' at depth 2), depth-1 string starts
struct Counts {
    uint32_t num, row, key, _pad;
};
struct Entry {          // state at a chunk's first byte
    int32_t state, depth;
};
// error word: (code << 48) | byte position (the minimum over the failures)
enum : uint64_t {
    kErrNone = 0,
    kErrNumber = 1,      // malformed number token
    kErrOverflow = 2,    // significand beyond u64
    kErrRange = 3,       // |value| past f64
    kErrSeparator = 4,   // a number not between '[' / ',' / ':' and ',' / ']' / '}'
    kErrDepth = 5,       // a number of m / u / v / d at the wrong nesting depth
    kErrRagged = 6,      // matrix rows of different lengths
};

hipError_t launch_pass1(const uint8_t* text, uint64_t n, Xfer* chunk_x, hipStream_t st);
hipError_t launch_scan1(const Xfer* chunk_x, uint32_t nchunks, Entry* entry, hipStream_t st);
hipError_t launch_pass2(const uint8_t* text, uint64_t n, const Entry* entry, Counts* chunk_c,
                        hipStream_t st);
// exclusive scan of the chunk counts in place; totals at chunk_c[nchunks]
hipError_t launch_scan2(Counts* chunk_c, uint32_t nchunks, hipStream_t st);
hipError_t launch_pass3(const uint8_t* text, uint64_t n, const Entry* entry, const Counts* chunk_off,
                        const double* pow10, double* val, uint64_t* npos, uint8_t* ndepth,
                        uint64_t* rpos, uint64_t* kpos, unsigned long long* err, hipStream_t st);
// out[2q] = lower_bound(npos, q-th query), out[2q + 1] = lower_bound(rpos, q-th query)
hipError_t launch_ranges(const uint64_t* npos, uint32_t nn, const uint64_t* rpos, uint32_t nr,
                         const uint64_t* queries, uint32_t nq, uint32_t* out, hipStream_t st);
// numbers [lo, hi) all at `depth`; matrix (rows > 0): row r (open at rpos[r0 + r])
// starts at number lo + r * cols
hipError_t launch_validate(const uint8_t* ndepth, uint32_t lo, uint32_t hi, uint32_t depth,
                           const uint64_t* npos, uint32_t nn, const uint64_t* rpos, uint32_t r0,
                           uint32_t rows, uint32_t cols, unsigned long long* err, hipStream_t st);

}  // namespace svdw_ingest_dev

// the interaction files parsed on the GPU.
//
// Reference: Loader.__init__ (code/dataloader.py:247-277) and the TF Data loader
// (LightGCN-tf/utility/load_data.py:27-48) read "uid item item ..." lines with Python loops.  Here
// the file's bytes go to the device once and two passes turn them into
//   line_user [n_lines]      the first number of every line that holds a number
//   line_ptr  [n_lines + 1]  CSR offsets of each line's remaining numbers (the items)
//   items     [n_pairs]      the items, in file order
//   pair_user [n_pairs]      the user of every item (optional) -- the reference's trainUser/trainItem
// A number is a maximal run of decimal digits; every other byte (space, tab, '\r', ...) separates
// numbers and '\n' ends a line, so "\r\n" endings, trailing spaces and a missing final newline are
// accepted.  Values must fit int32 (larger ones saturate).  Lines with no number are skipped.
//
// Layout: 64-KiB chunks (one 256-thread workgroup, 256 bytes per thread), staged in LDS by
// coalesced loads (per-thread byte walks over global memory ran at 25 GB/s).  Pass 1 counts the
// numbers and line-first numbers of every chunk; one workgroup scans the chunk counts (64-bit
// offsets: files beyond 2^31 bytes are fine); pass 2 recounts per thread, scans inside the
// workgroup and writes every number at its global position.  A number belongs to the chunk that
// holds its first digit and may end in the next.
#include "lgx_common.h"

namespace lgx {
namespace {

constexpr int kParseThreads = 256;
constexpr int64_t kBytesPerThread = 256;
constexpr int64_t kChunkBytes = kParseThreads * kBytesPerThread;

__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }

// The workgroup's 64-KiB chunk staged in LDS by coalesced 16-B loads, each thread's 256-B range
// padded by 16 B so that the threads' byte walks fall on different banks; bytes outside the
// chunk (a number's tail in the next chunk, the look-back before it) come from global memory.
constexpr int kSegPad = 16;
constexpr int kChunkLds = (int)(kChunkBytes + (kChunkBytes / kBytesPerThread) * kSegPad);

struct Text {
    const uint8_t* __restrict__ g;
    const uint8_t* s;  // LDS image of [lo, hi)
    int64_t lo, hi;
    __device__ __forceinline__ uint8_t operator[](int64_t i) const {
        if (i >= lo && i < hi) {
            const int64_t o = i - lo;
            return s[o + (o / kBytesPerThread) * kSegPad];
        }
        return g[i];
    }
};

__device__ Text stage_chunk(const uint8_t* __restrict__ g, int64_t n, uint8_t* img) {
    const int64_t lo = min((int64_t)blockIdx.x * kChunkBytes, n), hi = min(lo + kChunkBytes, n);
    if (hi - lo == kChunkBytes && ((uintptr_t)g & 15) == 0) {
        for (int q = threadIdx.x; q < (int)(kChunkBytes / 16); q += kParseThreads) {
            const uint4 v = reinterpret_cast<const uint4*>(g + lo)[q];
            const int o = q * 16;
            *reinterpret_cast<uint4*>(img + o + (o / kBytesPerThread) * kSegPad) = v;
        }
    } else {
        for (int64_t o = threadIdx.x; o < hi - lo; o += kParseThreads) img[o + (o / kBytesPerThread) * kSegPad] = g[lo + o];
    }
    __syncthreads();
    return Text{g, img, lo, hi};
}

__device__ __forceinline__ bool starts_number(const Text& t, int64_t i) {
    return is_digit(t[i]) && (i == 0 || !is_digit(t[i - 1]));
}

// the number starting at i is the first of its line: nothing but separators back to '\n' or the start
__device__ __forceinline__ bool first_of_line(const Text& t, int64_t i) {
    for (int64_t j = i - 1; j >= 0; --j) {
        const uint8_t c = t[j];
        if (c == '\n') return true;
        if (is_digit(c)) return false;
    }
    return true;
}

__device__ __forceinline__ int32_t parse_number(const Text& t, int64_t i, int64_t n) {
    int64_t v = 0;
    for (; i < n && is_digit(t[i]); ++i) {
        v = v * 10 + (t[i] - '0');
        if (v > INT32_MAX) v = INT32_MAX;  // saturate (ids must fit int32)
    }
    return (int32_t)v;
}

struct ThreadCounts {
    int64_t numbers, firsts;
};

__device__ __forceinline__ ThreadCounts count_range(const Text& t, int64_t lo, int64_t hi) {
    ThreadCounts c{0, 0};
    for (int64_t i = lo; i < hi; ++i) {
        if (starts_number(t, i)) {
            ++c.numbers;
            c.firsts += first_of_line(t, i) ? 1 : 0;
        }
    }
    return c;
}

// exclusive scan of one int64 per thread inside the workgroup; returns the workgroup total
__device__ int64_t block_exclusive_scan(int64_t v, int64_t* sh, int64_t* out) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int off = 1; off < kParseThreads; off <<= 1) {  // Hillis-Steele over 256 entries
        const int64_t x = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += x;
        __syncthreads();
    }
    *out = sh[tid] - v;
    const int64_t total = sh[kParseThreads - 1];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(kParseThreads) void parse_count_kernel(const uint8_t* __restrict__ t, int64_t n,
                                                                   int64_t* __restrict__ chunk_numbers,
                                                                   int64_t* __restrict__ chunk_firsts) {
    __shared__ int64_t sh[kParseThreads];
    __shared__ __attribute__((aligned(16))) uint8_t img[kChunkLds];
    const Text tx = stage_chunk(t, n, img);
    const int64_t lo = blockIdx.x * kChunkBytes + threadIdx.x * kBytesPerThread;
    const ThreadCounts c = count_range(tx, min(lo, n), min(lo + kBytesPerThread, n));
    int64_t dummy;
    const int64_t tn = block_exclusive_scan(c.numbers, sh, &dummy);
    const int64_t tf = block_exclusive_scan(c.firsts, sh, &dummy);
    if (threadIdx.x == 0) {
        chunk_numbers[blockIdx.x] = tn;
        chunk_firsts[blockIdx.x] = tf;
    }
}

// one workgroup: exclusive offsets of the chunk counts in place, totals to counts_out[0..1]
__global__ __launch_bounds__(kParseThreads) void parse_scan_kernel(int64_t* __restrict__ chunk_numbers,
                                                                  int64_t* __restrict__ chunk_firsts,
                                                                  int64_t n_chunks, int64_t* __restrict__ counts_out) {
    __shared__ int64_t sh[kParseThreads];
    const int64_t per = (n_chunks + kParseThreads - 1) / kParseThreads;
    const int64_t lo = min((int64_t)threadIdx.x * per, n_chunks), hi = min(lo + per, n_chunks);
    for (int a = 0; a < 2; ++a) {
        int64_t* c = a == 0 ? chunk_numbers : chunk_firsts;
        int64_t s = 0;
        for (int64_t i = lo; i < hi; ++i) s += c[i];
        int64_t base;
        const int64_t total = block_exclusive_scan(s, sh, &base);
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t x = c[i];
            c[i] = base;
            base += x;
        }
        if (threadIdx.x == 0) counts_out[a] = total;
    }
}

__global__ __launch_bounds__(kParseThreads) void parse_fill_kernel(const uint8_t* __restrict__ t, int64_t n,
                                                                  const int64_t* __restrict__ chunk_numbers,
                                                                  const int64_t* __restrict__ chunk_firsts,
                                                                  int32_t* __restrict__ line_user,
                                                                  int64_t* __restrict__ line_ptr,
                                                                  int32_t* __restrict__ items) {
    __shared__ int64_t sh[kParseThreads];
    __shared__ __attribute__((aligned(16))) uint8_t img[kChunkLds];
    const Text tx = stage_chunk(t, n, img);
    const int64_t lo = min(blockIdx.x * kChunkBytes + threadIdx.x * kBytesPerThread, n);
    const int64_t hi = min(lo + kBytesPerThread, n);
    const ThreadCounts c = count_range(tx, lo, hi);
    int64_t num_off, first_off;
    block_exclusive_scan(c.numbers, sh, &num_off);
    block_exclusive_scan(c.firsts, sh, &first_off);
    int64_t tok = chunk_numbers[blockIdx.x] + num_off;      // global index of this thread's next number
    int64_t lines = chunk_firsts[blockIdx.x] + first_off;   // line-first numbers before it
    for (int64_t i = lo; i < hi; ++i) {
        if (!starts_number(tx, i)) continue;
        const int32_t v = parse_number(tx, i, n);
        if (first_of_line(tx, i)) {
            line_user[lines] = v;
            line_ptr[lines] = tok - lines;  // items before this line
            ++lines;
        } else {
            items[tok - lines] = v;  // lines >= 1 here: a non-first number follows its line's first
        }
        ++tok;
    }
}

__global__ void parse_pair_user_kernel(const int32_t* __restrict__ line_user, const int64_t* __restrict__ line_ptr,
                                       int64_t n_lines, int32_t* __restrict__ pair_user) {
    const int64_t l = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (l >= n_lines) return;
    const int32_t u = line_user[l];
    for (int64_t p = line_ptr[l]; p < line_ptr[l + 1]; ++p) pair_user[p] = u;
}

__global__ void parse_close_kernel(int64_t* __restrict__ line_ptr, int64_t n_lines, int64_t n_pairs) {
    line_ptr[n_lines] = n_pairs;
}

int64_t n_chunks_of(int64_t n_bytes) { return n_bytes == 0 ? 0 : ceil_div(n_bytes, kChunkBytes); }

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_parse_lines_workspace(int64_t n_bytes, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && n_bytes >= 0, LGX_ERR_INVALID_ARG, "lgx_parse_lines_workspace: bad arguments");
    *ws_bytes = align_up((size_t)n_chunks_of(n_bytes) * 8) * 2 + 256;
    return LGX_OK;
}

extern "C" int lgx_parse_lines_count(const uint8_t* text, int64_t n_bytes, void* ws, size_t ws_bytes,
                                     int64_t* counts_out, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    size_t need = 0;
    lgx_parse_lines_workspace(n_bytes, &need);
    LGX_REQUIRE(n_bytes >= 0 && counts_out && (n_bytes == 0 || text), LGX_ERR_INVALID_ARG,
                "lgx_parse_lines_count: bad arguments");
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_parse_lines_count: workspace %zu < %zu", ws_bytes,
                need);
    const int64_t nc = n_chunks_of(n_bytes);
    int64_t* cn = static_cast<int64_t*>(ws);
    int64_t* cf = reinterpret_cast<int64_t*>(static_cast<char*>(ws) + align_up((size_t)nc * 8));
    if (nc > 0) {
        parse_count_kernel<<<(unsigned)nc, kParseThreads, 0, stream>>>(text, n_bytes, cn, cf);
        LGX_LAUNCH_CHECK();
    }
    parse_scan_kernel<<<1, kParseThreads, 0, stream>>>(cn, cf, nc, counts_out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_parse_lines_fill(const uint8_t* text, int64_t n_bytes, const void* ws, size_t ws_bytes,
                                    int64_t n_numbers, int64_t n_lines, int32_t* line_user, int64_t* line_ptr,
                                    int32_t* items, int32_t* pair_user, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    size_t need = 0;
    lgx_parse_lines_workspace(n_bytes, &need);
    LGX_REQUIRE(n_bytes >= 0 && n_lines >= 0 && n_numbers >= n_lines && line_ptr, LGX_ERR_INVALID_ARG,
                "lgx_parse_lines_fill: bad arguments");
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_parse_lines_fill: workspace %zu < %zu", ws_bytes, need);
    const int64_t n_pairs = n_numbers - n_lines;
    LGX_REQUIRE((n_lines == 0 || line_user) && (n_pairs == 0 || items), LGX_ERR_INVALID_ARG,
                "lgx_parse_lines_fill: missing output buffer");
    const int64_t nc = n_chunks_of(n_bytes);
    const int64_t* cn = static_cast<const int64_t*>(ws);
    const int64_t* cf = reinterpret_cast<const int64_t*>(static_cast<const char*>(ws) + align_up((size_t)nc * 8));
    if (nc > 0) {
        parse_fill_kernel<<<(unsigned)nc, kParseThreads, 0, stream>>>(text, n_bytes, cn, cf, line_user, line_ptr, items);
        LGX_LAUNCH_CHECK();
    }
    parse_close_kernel<<<1, 1, 0, stream>>>(line_ptr, n_lines, n_pairs);
    LGX_LAUNCH_CHECK();
    if (pair_user && n_lines > 0) {
        parse_pair_user_kernel<<<(unsigned)ceil_div(n_lines, (int64_t)256), 256, 0, stream>>>(line_user, line_ptr,
                                                                                            n_lines, pair_user);
        LGX_LAUNCH_CHECK();
    }
    return LGX_OK;
}

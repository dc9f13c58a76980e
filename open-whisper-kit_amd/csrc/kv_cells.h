// Self-attention KV cell bookkeeping of one clip, mirroring the reference's unified
// cache allocator (whisper_kv_cache_find_slot / _cell_max / _clear / _seq_rm / _seq_cp,
// ref src/whisper.cpp:968-1137). Only the cell <-> (position, sequence set) map lives
// here; the K/V rows themselves are in the engine's device cache. Reproducing the
// allocator matters for parity: the reference flash-attention visits the visible cells
// in cell order, and its F16 accumulator makes the result order-dependent.
#pragma once

#include <cstdint>
#include <limits>
#include <vector>

namespace owk {

struct KvCells {
    uint32_t head = 0, size = 0, n = 0;
    std::vector<int32_t> pos;
    std::vector<uint32_t> seq;  // bit s set <=> sequence s owns the cell (s < 32)

    void init(uint32_t n_ctx) {
        head = 0;
        size = n_ctx;
        pos.assign(n_ctx, -1);
        seq.assign(n_ctx, 0u);
    }
    void clear() {
        for (uint32_t i = 0; i < size; ++i) { pos[i] = -1; seq[i] = 0; }
        head = 0;
    }
    // contiguous slot for n_tokens tokens; returns the first cell or -1
    int find_slot(int n_tokens, const int32_t * tpos, const int32_t * tseq) {
        if ((uint32_t) n_tokens > size) return -1;
        uint32_t n_tested = 0;
        for (;;) {
            if (head + n_tokens > size) {
                n_tested += size - head;
                head = 0;
                continue;
            }
            bool found = true;
            for (int i = 0; i < n_tokens; ++i) {
                if (pos[head + i] >= 0) {
                    found = false;
                    head += i + 1;
                    n_tested += i + 1;
                    break;
                }
            }
            if (found) break;
            if (n_tested >= size) return -1;
        }
        for (int i = 0; i < n_tokens; ++i) {
            pos[head + i] = tpos[i];
            seq[head + i] |= 1u << tseq[i];
        }
        return (int) head;
    }
    int32_t cell_max() const {
        for (uint32_t i = size - 1; i > 0; --i)
            if (pos[i] >= 0 && seq[i] != 0) return (int32_t) i + 1;
        return 1;
    }
    void seq_rm(int s, int32_t p0, int32_t p1) {
        uint32_t new_head = size;
        if (p0 < 0) p0 = 0;
        if (p1 < 0) p1 = std::numeric_limits<int32_t>::max();
        for (uint32_t i = 0; i < size; ++i) {
            if (pos[i] >= p0 && pos[i] < p1) {
                if (s < 0) seq[i] = 0;
                else if (seq[i] & (1u << s)) seq[i] &= ~(1u << s);
                else continue;
                if (seq[i] == 0) {
                    pos[i] = -1;
                    if (new_head == size) new_head = i;
                }
            }
        }
        if (new_head != size) head = new_head;
    }
    void seq_cp(int src, int dst, int32_t p0, int32_t p1) {
        if (p0 < 0) p0 = 0;
        if (p1 < 0) p1 = std::numeric_limits<int32_t>::max();
        head = 0;
        for (uint32_t i = 0; i < size; ++i)
            if ((seq[i] & (1u << src)) && pos[i] >= p0 && pos[i] < p1) seq[i] |= 1u << dst;
    }
    // cells visible to (s, p): owned by s with pos <= p, among the first n cells, in cell order
    void visible(int s, int32_t p, std::vector<int> & out) const {
        for (uint32_t i = 0; i < n; ++i)
            if ((seq[i] & (1u << s)) && pos[i] <= p) out.push_back((int) i);
    }
};

} // namespace owk

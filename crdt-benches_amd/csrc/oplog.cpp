// oplog.cpp — order-statistic resolver over a chunked sequence (chunks of item ids + a Fenwick
// tree of per-chunk visible counts): O(log C + chunk) per positional lookup.
#include "oplog.hpp"

#include <algorithm>
#include <cstring>

#include "util.hpp"

namespace crdt {

namespace {
constexpr size_t kChunkMax = 512;
constexpr uint32_t kMagic = kUpdateMagic;
constexpr uint32_t kWireVersion = kUpdateVersion;

void put32(std::vector<uint8_t>& b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
uint32_t get32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
}  // namespace

OpLog::OpLog() { chunks_.emplace_back(); fen_build(); }

void OpLog::fen_build() {
    fen_.assign(chunks_.size() + 1, 0);
    for (size_t i = 0; i < chunks_.size(); ++i) {
        size_t j = i + 1;
        fen_[j] += chunks_[i].vis;
        size_t up = j + (j & (~j + 1));
        if (up <= chunks_.size()) fen_[up] += fen_[j];
    }
}

void OpLog::fen_add(size_t i, int64_t d) {
    for (size_t j = i + 1; j < fen_.size(); j += j & (~j + 1)) fen_[j] += d;
}

size_t OpLog::fen_find(uint64_t& p) const {
    size_t pos = 0;
    size_t step = 1;
    while (step * 2 < fen_.size()) step *= 2;
    for (; step; step >>= 1) {
        size_t nx = pos + step;
        if (nx < fen_.size() && (uint64_t)fen_[nx] < p) {
            pos = nx;
            p -= (uint64_t)fen_[nx];
        }
    }
    return pos;  // 0-based chunk; p is now the rank inside it
}

bool OpLog::find_visible(uint64_t p, size_t& c, size_t& i) const {
    if (p == 0 || p > nvis_) return false;
    uint64_t r = p;
    c = fen_find(r);
    if (c >= chunks_.size()) return false;
    const std::vector<uint32_t>& ids = chunks_[c].ids;
    for (i = 0; i < ids.size(); ++i) {
        if (!deleted[ids[i] - 1] && --r == 0) return true;
    }
    return false;
}

void OpLog::split_chunk(size_t c) {
    if (chunks_[c].ids.size() <= kChunkMax) return;
    std::vector<uint32_t> all;
    all.swap(chunks_[c].ids);
    size_t pieces = (all.size() + kChunkMax / 2 - 1) / (kChunkMax / 2);
    std::vector<Chunk> repl(pieces);
    for (size_t k = 0; k < pieces; ++k) {
        size_t a = k * all.size() / pieces, b = (k + 1) * all.size() / pieces;
        repl[k].ids.assign(all.begin() + a, all.begin() + b);
        for (uint32_t id : repl[k].ids) repl[k].vis += !deleted[id - 1];
    }
    chunks_.erase(chunks_.begin() + c);
    chunks_.insert(chunks_.begin() + c, repl.begin(), repl.end());
    fen_build();
}

std::string OpLog::insert(uint64_t pos, const uint32_t* cps, size_t k) {
    if (stale_) {
        std::string e = rebuild_index();
        if (!e.empty()) return e;
    }
    if (pos > nvis_) return "insert position out of range";
    if (k == 0) return "";
    if ((uint64_t)size() + k >= 0xFFFFFFF0ull) return "op log too large";
    size_t c = 0, at = 0;
    uint32_t left = 0;
    if (pos > 0) {
        size_t i;
        if (!find_visible(pos, c, i)) return "resolver index corrupt";
        left = chunks_[c].ids[i];
        at = i + 1;
    }
    // origin_right: the item now following `left` (tombstones included)
    uint32_t right = NIL;
    if (at < chunks_[c].ids.size()) {
        right = chunks_[c].ids[at];
    } else {
        for (size_t cc = c + 1; cc < chunks_.size(); ++cc)
            if (!chunks_[cc].ids.empty()) { right = chunks_[cc].ids[0]; break; }
    }
    uint32_t first = size() + 1;
    std::vector<uint32_t> ids(k);
    for (size_t j = 0; j < k; ++j) {
        uint32_t id = first + (uint32_t)j;
        parent.push_back(j == 0 ? left : id - 1);
        oright.push_back(right);
        lamport.push_back(++max_lamport);
        agent.push_back(local_agent);
        deleted.push_back(0);
        cp.push_back(cps[j]);
        ids[j] = id;
    }
    std::vector<uint32_t>& v = chunks_[c].ids;
    v.insert(v.begin() + at, ids.begin(), ids.end());
    chunks_[c].vis += (uint32_t)k;
    nvis_ += k;
    fen_add(c, (int64_t)k);
    split_chunk(c);
    return "";
}

std::string OpLog::insert_utf8(uint64_t pos, const char* s, size_t nbytes) {
    std::vector<uint32_t> cps;
    cps.reserve(nbytes);
    if (!utf8_decode(s, nbytes, cps)) return "invalid UTF-8";
    return insert(pos, cps.data(), cps.size());
}

std::string OpLog::remove(uint64_t start, uint64_t end) {
    if (stale_) {
        std::string e = rebuild_index();
        if (!e.empty()) return e;
    }
    if (end < start || end > nvis_) return "remove range out of range";
    uint64_t left = end - start;
    if (!left) return "";
    size_t c, i;
    if (!find_visible(start + 1, c, i)) return "resolver index corrupt";
    while (left) {
        if (i >= chunks_[c].ids.size()) { ++c; i = 0; continue; }
        uint32_t id = chunks_[c].ids[i++];
        if (deleted[id - 1]) continue;
        deleted[id - 1] = 1;
        del_ops.push_back(id);
        chunks_[c].vis--;
        fen_add(c, -1);
        --left;
    }
    nvis_ -= end - start;
    return "";
}

void OpLog::push_item(uint32_t par, uint32_t orr, uint32_t lam, uint16_t ag, uint8_t del,
                      uint32_t c) {
    parent.push_back(par);
    oright.push_back(orr);
    lamport.push_back(lam);
    agent.push_back(ag);
    deleted.push_back(del);
    cp.push_back(c);
    if (lam > max_lamport) max_lamport = lam;
    nvis_ += !del;
    stale_ = true;
}

void OpLog::mark_deleted(uint32_t id) {
    if (id == 0 || id > size() || deleted[id - 1]) return;
    deleted[id - 1] = 1;
    nvis_--;
    stale_ = true;
}

// Rebuild the positional index from the op log itself (RGA document order) after remote
// items arrived.  Host resolver bookkeeping only: merged documents always come from the device.
std::string OpLog::rebuild_index() {
    uint32_t n = size();
    std::vector<uint32_t> start(n + 2, 0), kids(n);
    for (uint32_t i = 1; i <= n; ++i) {
        uint32_t p = parent[i - 1];
        if (p > n || p == i) return "malformed op log (parent out of range)";
        start[p + 1]++;
    }
    for (uint32_t v = 0; v <= n; ++v) start[v + 1] += start[v];
    {
        std::vector<uint32_t> fill(start.begin(), start.end() - 1);
        for (uint32_t i = 1; i <= n; ++i) kids[fill[parent[i - 1]]++] = i;
    }
    auto newer = [&](uint32_t a, uint32_t b) {  // a sorts before b (greater timestamp first)
        if (lamport[a - 1] != lamport[b - 1]) return lamport[a - 1] > lamport[b - 1];
        return agent[a - 1] > agent[b - 1];
    };
    chunks_.clear();
    chunks_.emplace_back();
    nvis_ = 0;
    std::vector<uint32_t> stack;
    stack.reserve(n + 1);
    stack.push_back(0);
    size_t seen = 0;
    while (!stack.empty()) {
        uint32_t v = stack.back();
        stack.pop_back();
        if (v) {
            ++seen;
            if (chunks_.back().ids.size() >= kChunkMax / 2) chunks_.emplace_back();
            chunks_.back().ids.push_back(v);
            if (!deleted[v - 1]) { chunks_.back().vis++; nvis_++; }
        }
        uint32_t a = start[v], b = start[v + 1];
        std::sort(kids.begin() + a, kids.begin() + b, [&](uint32_t x, uint32_t y) { return newer(y, x); });
        for (uint32_t j = a; j < b; ++j) stack.push_back(kids[j]);  // oldest pushed first
    }
    if (seen != n) return "malformed op log (cycle)";
    fen_build();
    stale_ = false;
    return "";
}

// Wire format (little-endian): magic, version, first_id, n_items, first_del, n_dels,
// parent[n], origin_right[n], lamport[n], cp[n] (u32), agent[n] (u16, padded to 4), dels[m].
std::vector<uint8_t> OpLog::encode_from(uint64_t ver) const {
    uint32_t from_items = (uint32_t)(ver >> 32), from_dels = (uint32_t)ver;
    if (from_items > size()) from_items = size();
    if (from_dels > del_ops.size()) from_dels = (uint32_t)del_ops.size();
    uint32_t n = size() - from_items, m = (uint32_t)del_ops.size() - from_dels;
    std::vector<uint8_t> b;
    b.reserve(24 + (size_t)n * 18 + 4 + (size_t)m * 4);
    put32(b, kMagic);
    put32(b, kWireVersion);
    put32(b, from_items + 1);
    put32(b, n);
    put32(b, from_dels);
    put32(b, m);
    for (uint32_t k = 0; k < n; ++k) put32(b, parent[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) put32(b, oright[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) put32(b, lamport[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) put32(b, cp[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) {
        b.push_back((uint8_t)agent[from_items + k]);
        b.push_back((uint8_t)(agent[from_items + k] >> 8));
    }
    while (b.size() % 4) b.push_back(0);
    for (uint32_t k = 0; k < m; ++k) put32(b, del_ops[from_dels + k]);
    return b;
}

std::string OpLog::apply_update(const uint8_t* buf, size_t len) {
    if (len < 24 || get32(buf) != kMagic) return "not an update";
    if (get32(buf + 4) != kWireVersion) return "unsupported update version";
    uint32_t first = get32(buf + 8), n = get32(buf + 12);
    uint32_t first_del = get32(buf + 16), m = get32(buf + 20);
    size_t agent_bytes = ((size_t)n * 2 + 3) / 4 * 4;
    size_t need = 24 + (size_t)n * 16 + agent_bytes + (size_t)m * 4;
    if (len < need) return "truncated update";
    if (first == 0 || first > size() + 1) return "update is not causally ready (missing items)";
    const uint8_t* P = buf + 24;
    const uint8_t* O = P + (size_t)n * 4;
    const uint8_t* L = O + (size_t)n * 4;
    const uint8_t* C = L + (size_t)n * 4;
    const uint8_t* A = C + (size_t)n * 4;
    const uint8_t* D = A + agent_bytes;
    for (uint32_t k = 0; k < n; ++k) {
        uint32_t id = first + k;
        if (id <= size()) continue;  // already known (decode_and_add is idempotent)
        uint32_t par = get32(P + 4 * k);
        if (par >= id && par != 0) return "update item references an unknown parent";
        push_item(par, get32(O + 4 * k), get32(L + 4 * k),
                  (uint16_t)(A[2 * k] | (A[2 * k + 1] << 8)), 0, get32(C + 4 * k));
    }
    for (uint32_t k = 0; k < m; ++k) {
        uint32_t id = get32(D + 4 * k);
        if (id == 0 || id > size()) return "update deletes an unknown item";
        if (first_del + k >= del_ops.size()) del_ops.push_back(id);
        mark_deleted(id);
    }
    return "";
}

}  // namespace crdt

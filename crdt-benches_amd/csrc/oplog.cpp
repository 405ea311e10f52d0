// oplog.cpp — order-statistic resolver over a chunked span sequence (runs of consecutive ids,
// chunks of <= 64 spans + a Fenwick tree of per-chunk visible counts): O(log C + 64) per
// positional lookup, O(1) amortised appends while typing on (the span of the last item grows).
// A chunk hint and a span hint make the lookup of an edit next to the previous one O(1); the
// Fenwick tree is rebuilt only when a lookup misses the hints after chunks were split.
#include "oplog.hpp"

#include <algorithm>
#include <cstring>

#include "util.hpp"

namespace crdt {

namespace {
constexpr size_t kSpanMax = 64;
constexpr uint32_t kMagic = kUpdateMagic;
constexpr uint32_t kWireVersion = kUpdateVersion;

void put32(std::vector<uint8_t>& b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
uint32_t get32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
}  // namespace

OpLog::OpLog() {
    chunks_.push_back(new_chunk());
    fen_build();
    nxt_.push_back(NIL);
}

void OpLog::reserve(size_t items, size_t dels) {
    del_ops.reserve(dels);
    parent.reserve(items);
    oright.reserve(items);
    lamport.reserve(items);
    cp.reserve(items);
    agent.reserve(items);
    deleted.reserve(items);
    nxt_.reserve(items + 1);
}

OpLog::Chunk OpLog::new_chunk() const {
    Chunk c;
    c.s.reserve(kSpanMax + 4);
    return c;
}

void OpLog::fen_build() const {
    fen_dirty_ = false;
    fen_.assign(chunks_.size() + 1, 0);
    for (size_t i = 0; i < chunks_.size(); ++i) {
        size_t j = i + 1;
        fen_[j] += chunks_[i].vis;
        size_t up = j + (j & (~j + 1));
        if (up <= chunks_.size()) fen_[up] += fen_[j];
    }
}

void OpLog::fen_add(size_t i, int64_t d) {
    if (fen_dirty_) return;  // (the rebuild counts the chunks as they are then)
    for (size_t j = i + 1; j < fen_.size(); j += j & (~j + 1)) fen_[j] += d;
}

size_t OpLog::fen_find(uint64_t& p) const {
    if (fen_dirty_) fen_build();
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

bool OpLog::find_visible(uint64_t p, size_t& c, size_t& si, uint32_t& off) const {
    if (p == 0 || p > nvis_) return false;
    uint64_t r = p;
    if (hint_c_ < chunks_.size() && p > hint_base_ && p - hint_base_ <= chunks_[hint_c_].vis) {
        c = hint_c_;
        r = p - hint_base_;
    } else {
        c = fen_find(r);
        if (c >= chunks_.size()) return false;
        hint_c_ = c;
        hint_base_ = p - r;
        hint_si_ = SIZE_MAX;
    }
    const std::vector<Span>& v = chunks_[c].s;
    si = 0;
    uint64_t vb = 0;  // visible items of the chunk before span si
    if (hint_si_ < v.size() && r > hint_vb_) {
        si = hint_si_;
        vb = hint_vb_;
    }
    for (; si < v.size(); ++si) {
        if (v[si].del()) continue;
        const uint32_t len = v[si].len();
        if (r - vb <= len) {
            off = (uint32_t)(r - vb) - 1;
            hint_si_ = si;
            hint_vb_ = vb;
            return true;
        }
        vb += len;
    }
    return false;
}

uint32_t OpLog::first_id_from(size_t c, size_t si) const {
    for (; c < chunks_.size(); ++c, si = 0)
        if (si < chunks_[c].s.size()) return chunks_[c].s[si].id;
    return NIL;
}

bool OpLog::split_chunk(size_t c) {
    if (chunks_[c].s.size() <= kSpanMax) return false;
    Chunk hi = new_chunk();
    std::vector<Span>& lo = chunks_[c].s;
    size_t half = lo.size() / 2;
    hi.s.assign(lo.begin() + half, lo.end());
    lo.resize(half);
    for (const Span& x : hi.s)
        if (!x.del()) hi.vis += x.len();
    chunks_[c].vis -= hi.vis;
    chunks_.insert(chunks_.begin() + c + 1, std::move(hi));
    fen_dirty_ = true;
    if (hint_c_ == c && hint_si_ >= half) hint_si_ = SIZE_MAX;  // the span moved to chunk c + 1
    if (hint_c_ != SIZE_MAX && hint_c_ > c) hint_c_++;         // (its visible base is unchanged)
    return true;
}

std::string OpLog::insert(uint64_t pos, const uint32_t* cps, size_t k) {
    if (stale_) {
        std::string e = rebuild_index();
        if (!e.empty()) return e;
    }
    if (!fugue) return insert_rga(pos, cps, k);
    if (pos > nvis_) return "insert position out of range";
    if (k == 0) return "";
    if ((uint64_t)size() + k >= 0x7FFFFFF0ull) return "op log too large";
    const uint32_t first = size() + 1;
    size_t c = 0, at = 0;  // new span goes to chunks_[c].s[at]
    uint32_t left = 0, right;
    bool extend = false;
    if (pos == 0) {
        right = first_id_from(0, 0);
        hint_c_ = 0;  // chunk 0 changes: keep the hint on it
        hint_base_ = 0;
        hint_si_ = SIZE_MAX;
    } else {
        size_t si;
        uint32_t off;
        if (!find_visible(pos, c, si, off)) return "resolver index corrupt";
        std::vector<Span>& v = chunks_[c].s;
        const Span S = v[si];
        left = S.id + off;
        if (off + 1 < S.len()) {  // split S after `left`
            right = left + 1;
            v[si].n = off + 1;
            v.insert(v.begin() + si + 1, Span{left + 1, S.len() - off - 1});
        } else {
            right = first_id_from(c, si + 1);
            extend = (S.id + S.len() == first);  // typing on: left is the last item created
        }
        at = si + 1;
    }
    if (fugue) {  // Fugue anchors (see oplog.hpp); every char after the first is a right child
        if (hasright_.size() < (size_t)first + k) hasright_.resize(std::max<size_t>(first + k, 2 * hasright_.size()), 0);
        const bool as_left = hasright_[left] != 0;
        if (as_left && right == NIL) return "resolver index corrupt (Fugue: no right neighbour)";
        side.resize(side.size() + k, 0);
        side[first - 1] = as_left ? 1 : 0;
        if (!as_left) hasright_[left] = 1;
        for (size_t j = 1; j < k; ++j) hasright_[first + j - 1] = 1;
        if (k == 1) {
            parent.push_back(as_left ? right : left);
            oright.push_back(right);
            lamport.push_back(++max_lamport);
            agent.push_back(local_agent);
            deleted.push_back(0);
            cp.push_back(cps[0]);
        } else {
            const size_t n0 = parent.size();
            parent.resize(n0 + k);
            oright.resize(n0 + k, right);
            lamport.resize(n0 + k);
            agent.resize(n0 + k, local_agent);
            deleted.resize(n0 + k, 0);
            cp.resize(n0 + k);
            parent[n0] = as_left ? right : left;
            for (size_t j = 1; j < k; ++j) parent[n0 + j] = first + (uint32_t)j - 1;
            for (size_t j = 0; j < k; ++j) lamport[n0 + j] = max_lamport + 1 + (uint32_t)j;
            max_lamport += (uint32_t)k;
            std::memcpy(cp.data() + n0, cps, k * sizeof(uint32_t));
        }
    } else if (k == 1) {  // typing: one item
        parent.push_back(left);
        oright.push_back(right);
        lamport.push_back(++max_lamport);
        agent.push_back(local_agent);
        deleted.push_back(0);
        cp.push_back(cps[0]);
    } else {  // a paste: every column grown once, then filled
        const size_t n0 = parent.size();
        parent.resize(n0 + k);
        oright.resize(n0 + k);
        lamport.resize(n0 + k);
        agent.resize(n0 + k, local_agent);
        deleted.resize(n0 + k, 0);
        cp.resize(n0 + k);
        uint32_t* P = parent.data() + n0;
        uint32_t* O = oright.data() + n0;
        uint32_t* L = lamport.data() + n0;
        P[0] = left;
        for (size_t j = 1; j < k; ++j) P[j] = first + (uint32_t)j - 1;
        for (size_t j = 0; j < k; ++j) {
            O[j] = right;
            L[j] = max_lamport + 1 + (uint32_t)j;
        }
        max_lamport += (uint32_t)k;
        std::memcpy(cp.data() + n0, cps, k * sizeof(uint32_t));
    }
    std::vector<Span>& v = chunks_[c].s;
    if (extend)
        v[at - 1].n += (uint32_t)k;
    else
        v.insert(v.begin() + at, Span{first, (uint32_t)k});
    chunks_[c].vis += (uint32_t)k;
    nvis_ += k;
    fen_add(c, (int64_t)k);
    split_chunk(c);
    return "";
}

// ---- RGA: gap buffer of visible id spans + full-list successors --------------------------------
void OpLog::gb_move(uint64_t pos) {
    while (gvis_ > pos) {
        GSpan& sp = gb_[g0_ - 1];
        if (gvis_ - sp.len >= pos) {
            gb_[--g1_] = sp;
            --g0_;
            gvis_ -= sp.len;
        } else {  // split: the part after pos goes right of the gap
            const uint32_t o = (uint32_t)(pos - (gvis_ - sp.len));
            gb_[--g1_] = GSpan{sp.id + o, sp.len - o};
            sp.len = o;
            gvis_ = pos;
        }
    }
    while (gvis_ < pos) {
        GSpan& sp = gb_[g1_];
        if (gvis_ + sp.len <= pos) {
            gb_[g0_++] = sp;
            ++g1_;
            gvis_ += sp.len;
        } else {
            const uint32_t o = (uint32_t)(pos - gvis_);
            gb_[g0_++] = GSpan{sp.id, o};
            sp.id += o;
            sp.len -= o;
            gvis_ = pos;
        }
    }
}

void OpLog::gb_reserve(size_t k) {
    if (g1_ - g0_ >= k) return;
    const size_t tail = gb_.size() - g1_;
    const size_t cap = std::max<size_t>({2 * gb_.size(), gb_.size() + k + 64, 1024});
    gb_.resize(cap);
    std::memmove(gb_.data() + cap - tail, gb_.data() + g1_, tail * sizeof(GSpan));
    g1_ = cap - tail;
}

std::string OpLog::insert_rga(uint64_t pos, const uint32_t* cps, size_t k) {
    if (pos > nvis_) return "insert position out of range";
    if (k == 0) return "";
    if ((uint64_t)size() + k >= 0x7FFFFFF0ull) return "op log too large";
    const uint32_t first = size() + 1;
    gb_reserve(2);  // (a split and a new span)
    gb_move(pos);
    // origin_left: the pos-th visible item, the last one before the gap
    const uint32_t left = pos ? gb_[g0_ - 1].id + gb_[g0_ - 1].len - 1u : 0u;
    const uint32_t right = nxt_[left];  // origin_right (tombstones included)
    // the new items follow left in the full list, before whatever followed it
    nxt_[left] = first;
    const size_t n0 = parent.size();
    if (k == 1) {  // typing: one item
        parent.push_back(left);
        oright.push_back(right);
        lamport.push_back(++max_lamport);
        agent.push_back(local_agent);
        deleted.push_back(0);
        cp.push_back(cps[0]);
        nxt_.push_back(right);
    } else {  // a paste: every column grown once, then filled
        parent.resize(n0 + k);
        oright.resize(n0 + k, right);
        lamport.resize(n0 + k);
        agent.resize(n0 + k, local_agent);
        deleted.resize(n0 + k, 0);
        cp.resize(n0 + k);
        nxt_.resize(n0 + 1 + k);
        uint32_t* P = parent.data() + n0;
        uint32_t* L = lamport.data() + n0;
        uint32_t* N = nxt_.data() + n0 + 1;
        P[0] = left;
        for (size_t j = 1; j < k; ++j) P[j] = first + (uint32_t)j - 1;
        for (size_t j = 0; j < k; ++j) {
            L[j] = max_lamport + 1 + (uint32_t)j;
            N[j] = first + (uint32_t)j + 1;
        }
        N[k - 1] = right;
        max_lamport += (uint32_t)k;
        std::memcpy(cp.data() + n0, cps, k * sizeof(uint32_t));
    }
    if (g0_ && gb_[g0_ - 1].id + gb_[g0_ - 1].len == first)
        gb_[g0_ - 1].len += (uint32_t)k;  // typing on: the span before the gap grows
    else
        gb_[g0_++] = GSpan{first, (uint32_t)k};
    gvis_ += k;
    nvis_ += k;
    return "";
}

std::string OpLog::remove_rga(uint64_t start, uint64_t end) {
    if (end < start || end > nvis_) return "remove range out of range";
    uint64_t left = end - start;
    if (!left) return "";
    gb_reserve(1);
    gb_move(start);
    nvis_ -= left;
    while (left) {  // the visible items right of the gap, span by span
        GSpan& sp = gb_[g1_];
        const uint32_t take = (uint32_t)std::min<uint64_t>(left, sp.len);
        const size_t m0 = del_ops.size();
        del_ops.resize(m0 + take);
        uint32_t* D = del_ops.data() + m0;
        for (uint32_t j = 0; j < take; ++j) D[j] = sp.id + j;
        std::memset(deleted.data() + sp.id - 1, 1, take);
        if (take == sp.len) {
            ++g1_;
        } else {
            sp.id += take;
            sp.len -= take;
        }
        left -= take;
    }
    return "";
}

// The resolver's hot loop for RGA logs (the upstream closure, main.rs:28-36).  The same steps as
// remove_rga + insert_rga, fused: every column is sized once to the trace's bound and written by
// index (no per-item push_back), a one-byte insert (typing) and a one-codepoint delete
// (backspace) take straight-line paths, and no std::string is made per patch.
std::string OpLog::replay(const uint64_t* pt, size_t np, const char* ins, size_t ins_total) {
    if (fugue || stale_) {
        for (size_t i = 0; i < np; ++i) {
            const uint64_t* q = pt + 4 * i;
            std::string e;
            if (q[1]) e = remove(q[0], q[0] + q[1]);
            if (e.empty() && q[3]) e = insert_utf8(q[0], ins + q[2], q[3]);
            if (!e.empty()) return e;
        }
        return "";
    }
    // bounds without a pass over the patches: items <= the inserted bytes, and every item is
    // deleted at most once (the columns are default-initialised: the slack costs no writes)
    size_t n = parent.size(), m = del_ops.size();
    const size_t ib = ins_total, db = n + ib;
    if ((uint64_t)n + ib >= 0x7FFFFFF0ull) return "op log too large";
    parent.resize(n + ib);
    oright.resize(n + ib);
    lamport.resize(n + ib);
    agent.resize(n + ib);
    deleted.resize(n + ib);
    cp.resize(n + ib);
    nxt_.resize(n + 1 + ib);
    del_ops.resize(m + db);
    uint32_t *P = parent.data(), *O = oright.data(), *L = lamport.data(), *C = cp.data();
    uint16_t* A = agent.data();
    uint8_t* Dl = deleted.data();
    uint32_t *N = nxt_.data(), *Do = del_ops.data();
    // the gap buffer's state and the counters in locals for the whole loop (the byte stores to
    // the deleted column may alias any member, which would reload them after every store)
    // (a patch adds at most three spans: a split at its delete, a split at its insert and the
    // new span; the gap buffer is default-initialised, so the room costs no writes)
    gb_reserve(3 * np + 64);
    GSpan* G = gb_.data();
    size_t g0 = g0_, g1 = g1_;
    uint64_t gvis = gvis_, nvis = nvis_;
    uint32_t maxl = max_lamport;
    const uint16_t agent0 = local_agent;
    // the gap to visible position pos (gb_move on the locals)
    auto move_to = [&](uint64_t pos) {
        while (gvis > pos) {
            GSpan& sp = G[g0 - 1];
            if (gvis - sp.len >= pos) {
                G[--g1] = sp;
                --g0;
                gvis -= sp.len;
            } else {  // split: the part after pos goes right of the gap
                const uint32_t o = (uint32_t)(pos - (gvis - sp.len));
                G[--g1] = GSpan{sp.id + o, sp.len - o};
                sp.len = o;
                gvis = pos;
            }
        }
        while (gvis < pos) {
            GSpan& sp = G[g1];
            if (gvis + sp.len <= pos) {
                G[g0++] = sp;
                ++g1;
                gvis += sp.len;
            } else {
                const uint32_t o = (uint32_t)(pos - gvis);
                G[g0++] = GSpan{sp.id, o};
                sp.id += o;
                sp.len -= o;
                gvis = pos;
            }
        }
    };
    const char* err = nullptr;
    for (size_t i = 0; i < np && !err; ++i) {
        const uint64_t pos = pt[4 * i], del = pt[4 * i + 1], ioff = pt[4 * i + 2], ilen = pt[4 * i + 3];
        if (del) {  // (remove_rga)
            if (pos + del > nvis) {
                err = "remove range out of range";
                break;
            }
            move_to(pos);
            nvis -= del;
            uint64_t left = del;
            while (left) {
                GSpan& sp = G[g1];
                const uint32_t take = (uint32_t)std::min<uint64_t>(left, sp.len);
                for (uint32_t j = 0; j < take; ++j) Do[m + j] = sp.id + j;
                m += take;
                std::memset(Dl + sp.id - 1, 1, take);
                if (take == sp.len) {
                    ++g1;
                } else {
                    sp.id += take;
                    sp.len -= take;
                }
                left -= take;
            }
        }
        if (!ilen) continue;
        // (insert_rga) the codepoints: one ASCII byte while typing, else decoded
        const unsigned char* s8 = reinterpret_cast<const unsigned char*>(ins + ioff);
        uint32_t c1;
        const uint32_t* cps;
        size_t k;
        if (ilen == 1 && s8[0] < 0x80u) {
            c1 = s8[0];
            cps = &c1;
            k = 1;
        } else {
            cps_.clear();
            if (!utf8_decode(reinterpret_cast<const char*>(s8), ilen, cps_)) {
                err = "invalid UTF-8";
                break;
            }
            cps = cps_.data();
            k = cps_.size();
        }
        if (pos > nvis) {
            err = "insert position out of range";
            break;
        }
        const uint32_t first = (uint32_t)n + 1;
        move_to(pos);
        const uint32_t lft = pos ? G[g0 - 1].id + G[g0 - 1].len - 1u : 0u;
        const uint32_t rgt = N[lft];
        N[lft] = first;
        if (k == 1) {  // (typing)
            P[n] = lft;
            O[n] = rgt;
            L[n] = maxl + 1u;
            A[n] = agent0;
            Dl[n] = 0;
            C[n] = cps[0];
        } else {  // (a paste: column by column, each loop vectorises)
            P[n] = lft;
            for (size_t j = 1; j < k; ++j) P[n + j] = first + (uint32_t)j - 1u;
            std::fill(O + n, O + n + k, rgt);
            for (size_t j = 0; j < k; ++j) L[n + j] = maxl + 1u + (uint32_t)j;
            std::fill(A + n, A + n + k, agent0);
            std::memset(Dl + n, 0, k);
            std::memcpy(C + n, cps, k * sizeof(uint32_t));
            for (size_t j = 0; j + 1 < k; ++j) N[n + 1 + j] = first + (uint32_t)j + 1u;
        }
        N[n + k] = rgt;
        maxl += (uint32_t)k;
        n += k;
        if (g0 && G[g0 - 1].id + G[g0 - 1].len == first)
            G[g0 - 1].len += (uint32_t)k;  // typing on: the span before the gap grows
        else
            G[g0++] = GSpan{first, (uint32_t)k};
        gvis += k;
        nvis += k;
    }
    g0_ = g0;
    g1_ = g1;
    gvis_ = gvis;
    nvis_ = nvis;
    max_lamport = maxl;
    parent.resize(n);
    oright.resize(n);
    lamport.resize(n);
    agent.resize(n);
    deleted.resize(n);
    cp.resize(n);
    nxt_.resize(n + 1);
    del_ops.resize(m);
    return err ? std::string(err) : std::string();
}

// The gap buffer and the successors from the full document order (ids, tombstones included).
std::string OpLog::rebuild_index_rga(const std::vector<uint32_t>& order) {
    nxt_.assign((size_t)size() + 1, NIL);
    gb_.assign(1024, GSpan{0, 0});
    g0_ = 0;
    g1_ = gb_.size();
    uint32_t prev = 0;
    uint64_t v = 0;
    for (uint32_t id : order) {
        nxt_[prev] = id;
        prev = id;
        if (deleted[id - 1]) continue;
        ++v;
        if (g0_ && gb_[g0_ - 1].id + gb_[g0_ - 1].len == id) {
            gb_[g0_ - 1].len++;
        } else {
            gb_reserve(1);
            gb_[g0_++] = GSpan{id, 1};
        }
    }
    gvis_ = v;
    nvis_ = v;
    stale_ = false;
    return "";
}

std::string OpLog::insert_utf8(uint64_t pos, const char* s, size_t nbytes) {
    if (nbytes == 1 && (unsigned char)s[0] < 0x80u) {  // typing one ASCII character
        const uint32_t c = (unsigned char)s[0];
        return insert(pos, &c, 1);
    }
    cps_.clear();
    if (!utf8_decode(s, nbytes, cps_)) return "invalid UTF-8";
    return insert(pos, cps_.data(), cps_.size());
}

// Tombstone items [off, off+take) of visible span si; merges the tombstone span with deleted
// neighbours whose ids continue it.  Returns the index of the span after the tombstones.
size_t OpLog::delete_in_span(Chunk& ch, size_t si, uint32_t off, uint32_t take) {
    std::vector<Span>& v = ch.s;
    const Span S = v[si];
    const uint32_t len = S.len(), did = S.id + off, dend = did + take;
    if (take == 1) {  // backspace
        deleted[did - 1] = 1;
        del_ops.push_back(did);
    } else {
        std::memset(deleted.data() + did - 1, 1, take);
        const size_t m0 = del_ops.size();
        del_ops.resize(m0 + take);
        for (uint32_t j = 0; j < take; ++j) del_ops[m0 + j] = did + j;
    }
    Span rep[3];
    int nr = 0;
    if (off) rep[nr++] = Span{S.id, off};
    size_t mid = si + nr;
    rep[nr++] = Span{did, take | 0x80000000u};
    const bool tail = off + take < len;
    if (tail) rep[nr++] = Span{dend, len - off - take};
    v[si] = rep[0];
    if (nr > 1) v.insert(v.begin() + si + 1, rep + 1, rep + nr);
    if (!tail && mid + 1 < v.size() && v[mid + 1].del() && v[mid + 1].id == dend) {
        v[mid].n += v[mid + 1].len();
        v.erase(v.begin() + mid + 1);
    }
    if (mid > 0 && v[mid - 1].del() && v[mid - 1].id + v[mid - 1].len() == did) {
        v[mid - 1].n += v[mid].len();
        v.erase(v.begin() + mid);
        --mid;
    }
    return mid + 1;
}

std::string OpLog::remove(uint64_t start, uint64_t end) {
    if (stale_) {
        std::string e = rebuild_index();
        if (!e.empty()) return e;
    }
    if (!fugue) return remove_rga(start, end);
    if (end < start || end > nvis_) return "remove range out of range";
    uint64_t left = end - start;
    if (!left) return "";
    size_t c, si;
    uint32_t off;
    if (!find_visible(start + 1, c, si, off)) return "resolver index corrupt";
    const size_t c0 = c;
    while (left) {
        Chunk& ch = chunks_[c];
        if (si >= ch.s.size()) {
            if (++c >= chunks_.size()) return "resolver index corrupt";
            si = 0;
            off = 0;
            continue;
        }
        if (ch.s[si].del()) {
            ++si;
            off = 0;
            continue;
        }
        uint32_t take = ch.s[si].len() - off;
        if (take > left) take = (uint32_t)left;
        si = delete_in_span(ch, si, off, take);
        off = 0;
        ch.vis -= take;
        fen_add(c, -(int64_t)take);
        left -= take;
    }
    nvis_ -= end - start;
    for (size_t cc = c + 1; cc-- > c0;) split_chunk(cc);
    return "";
}

void OpLog::push_item(uint32_t par, uint32_t orr, uint32_t lam, uint16_t ag, uint8_t del,
                      uint32_t c, uint8_t sd) {
    if (fugue) side.push_back(sd);
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
    if (fugue) return rebuild_index_fugue();
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
    std::vector<uint32_t> order;
    order.reserve(n);
    std::vector<uint32_t> stack;
    stack.reserve(n + 1);
    stack.push_back(0);
    while (!stack.empty()) {
        uint32_t v = stack.back();
        stack.pop_back();
        if (v) order.push_back(v);
        uint32_t a = start[v], b = start[v + 1];
        std::sort(kids.begin() + a, kids.begin() + b, [&](uint32_t x, uint32_t y) { return newer(y, x); });
        for (uint32_t j = a; j < b; ++j) stack.push_back(kids[j]);  // oldest pushed first
    }
    if (order.size() != n) return "malformed op log (cycle)";
    return rebuild_index_rga(order);
}

// Appends item v to the end of the rebuilt sequence.
void OpLog::index_append(uint32_t v) {
    const bool del = deleted[v - 1] != 0;
    Chunk* ch = &chunks_.back();
    Span* last = ch->s.empty() ? nullptr : &ch->s.back();
    if (last && last->del() == del && last->id + last->len() == v) {
        last->n++;
    } else {
        if (ch->s.size() >= kSpanMax / 2) {
            chunks_.push_back(new_chunk());
            ch = &chunks_.back();
        }
        ch->s.push_back(Span{v, 1u | (del ? 0x80000000u : 0u)});
    }
    if (!del) { ch->vis++; nvis_++; }
}

// The Fugue in-order (left children by timestamp descending, the item, then its right children
// by timestamp descending), as orc_merge_fugue (oracle/oracle.c) walks it; also recomputes
// hasright_ with the remote right children.
std::string OpLog::rebuild_index_fugue() {
    const uint32_t n = size();
    if (side.size() != n) return "malformed op log (side column)";
    std::vector<uint32_t> start(2ull * n + 3, 0), kids(n);  // groups 2v (left), 2v + 1 (right)
    for (uint32_t i = 1; i <= n; ++i) {
        const uint32_t p = parent[i - 1];
        if (p > n || p == i || (p == 0 && side[i - 1])) return "malformed op log (parent out of range)";
        start[2ull * p + (side[i - 1] ? 0 : 1) + 1]++;
    }
    for (uint64_t g = 0; g < 2ull * n + 2; ++g) start[g + 1] += start[g];
    {
        std::vector<uint32_t> fill(start.begin(), start.end() - 1);
        for (uint32_t i = 1; i <= n; ++i) kids[fill[2ull * parent[i - 1] + (side[i - 1] ? 0 : 1)]++] = i;
    }
    hasright_.assign(std::max<size_t>(hasright_.size(), (size_t)n + 1), 0);
    for (uint32_t i = 1; i <= n; ++i)
        if (!side[i - 1]) hasright_[parent[i - 1]] = 1;
    auto older = [&](uint32_t a, uint32_t b) {  // a has the smaller timestamp
        if (lamport[a - 1] != lamport[b - 1]) return lamport[a - 1] < lamport[b - 1];
        return agent[a - 1] < agent[b - 1];
    };
    chunks_.clear();
    chunks_.push_back(new_chunk());
    nvis_ = 0;
    hint_c_ = SIZE_MAX;
    hint_si_ = SIZE_MAX;
    constexpr uint32_t EMIT = 0x80000000u;
    std::vector<uint32_t> stack;
    stack.reserve(2ull * n + 2);
    stack.push_back(0);
    size_t seen = 0;
    while (!stack.empty()) {
        const uint32_t e = stack.back();
        stack.pop_back();
        if (e & EMIT) {
            ++seen;
            index_append(e & ~EMIT);
            continue;
        }
        // pushed in reverse of the walk: right children, e, left children (each oldest first)
        const uint32_t l0 = start[2ull * e], l1 = start[2ull * e + 1], r1 = start[2ull * e + 2];
        std::sort(kids.begin() + l0, kids.begin() + l1, older);
        std::sort(kids.begin() + l1, kids.begin() + r1, older);
        for (uint32_t j = l1; j < r1; ++j) stack.push_back(kids[j]);
        if (e) stack.push_back(e | EMIT);
        for (uint32_t j = l0; j < l1; ++j) stack.push_back(kids[j]);
    }
    if (seen != n) return "malformed op log (cycle)";
    fen_build();
    stale_ = false;
    return "";
}

// Wire format (little-endian): magic, version, first_id, n_items, first_del, n_dels,
// parent[n], origin_right[n], lamport[n], cp[n] (u32), agent[n] (u16, padded to 4), dels[m].
// Fugue logs write version 2, with bit 31 of cp[k] = side (1: left child of parent[k]).
std::vector<uint8_t> OpLog::encode_from(uint64_t ver) const {
    uint32_t from_items = (uint32_t)(ver >> 32), from_dels = (uint32_t)ver;
    if (from_items > size()) from_items = size();
    if (from_dels > del_ops.size()) from_dels = (uint32_t)del_ops.size();
    uint32_t n = size() - from_items, m = (uint32_t)del_ops.size() - from_dels;
    std::vector<uint8_t> b;
    b.reserve(24 + (size_t)n * 18 + 4 + (size_t)m * 4);
    put32(b, kMagic);
    put32(b, fugue ? kUpdateVersionFugue : kWireVersion);
    put32(b, from_items + 1);
    put32(b, n);
    put32(b, from_dels);
    put32(b, m);
    for (uint32_t k = 0; k < n; ++k) put32(b, parent[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) put32(b, oright[from_items + k]);
    for (uint32_t k = 0; k < n; ++k) put32(b, lamport[from_items + k]);
    if (fugue)
        for (uint32_t k = 0; k < n; ++k)
            put32(b, cp[from_items + k] | (side[from_items + k] ? kUpdateSideBit : 0u));
    else
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
    const uint32_t ver = get32(buf + 4);
    if (ver == kUpdateVersionFugue && !fugue) return "Fugue update into an RGA log";
    if (ver != kWireVersion && ver != kUpdateVersionFugue) return "unsupported update version";
    uint32_t first = get32(buf + 8), n = get32(buf + 12);
    uint32_t first_del = get32(buf + 16), m = get32(buf + 20);
    size_t agent_bytes = ((size_t)n * 2 + 3) / 4 * 4;
    size_t need = 24 + (size_t)n * 16 + agent_bytes + (size_t)m * 4;
    if (len < need) return "truncated update";
    if (first == 0 || first > size() + 1) return "update is not causally ready (missing items)";
    if (first_del > del_ops.size()) return "update is not causally ready (missing deletes)";
    if ((uint64_t)first + n > 0xFFFFFFFFull) return "update item ids out of range";
    const uint8_t* P = buf + 24;
    const uint8_t* O = P + (size_t)n * 4;
    const uint8_t* L = O + (size_t)n * 4;
    const uint8_t* C = L + (size_t)n * 4;
    const uint8_t* A = C + (size_t)n * 4;
    const uint8_t* D = A + agent_bytes;
    // validate everything before changing anything: a rejected update leaves the log as it was
    // (as the device decoder does with a rejected batch)
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t id = first + k, par = get32(P + 4 * k);
        if (id > size() && par >= id && par != 0) return "update item references an unknown parent";
        if (fugue && id > size()) {
            if (par == 0 && (get32(C + 4 * k) & kUpdateSideBit))
                return "update item is a left child of the document start";
            if (get32(L + 4 * k) == 0xFFFFFFFFu) return "Fugue update item with lamport 0xFFFFFFFF";
        }
    }
    const uint64_t known = std::max<uint64_t>(size(), n ? (uint64_t)first + n - 1 : 0);
    for (uint32_t k = 0; k < m; ++k) {
        const uint32_t id = get32(D + 4 * k);
        if (id == 0 || id > known) return "update deletes an unknown item";
    }
    for (uint32_t k = 0; k < n; ++k) {
        uint32_t id = first + k;
        if (id <= size()) continue;  // already known (decode_and_add is idempotent)
        const uint32_t c = get32(C + 4 * k);
        push_item(get32(P + 4 * k), get32(O + 4 * k), get32(L + 4 * k),
                  (uint16_t)(A[2 * k] | (A[2 * k + 1] << 8)), 0, c & ~kUpdateSideBit,
                  fugue && (c & kUpdateSideBit) ? 1 : 0);
    }
    for (uint32_t k = 0; k < m; ++k) {
        const uint32_t id = get32(D + 4 * k);
        if (first_del + k >= del_ops.size()) del_ops.push_back(id);
        mark_deleted(id);
    }
    return "";
}

}  // namespace crdt

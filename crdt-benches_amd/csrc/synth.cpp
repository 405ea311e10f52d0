// synth.cpp — synthetic anchor op logs, splitmix64-seeded.
#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "oplog.hpp"
#include "synth.hpp"
#include "util.hpp"

namespace crdt {

namespace {
// ~1% of items get a multi-byte codepoint so UTF-8 scatter paths are exercised.
uint32_t pick_cp(uint64_t h) {
    static const uint32_t wide[] = {0x00E9, 0x00F7, 0x0192, 0x2019, 0x2191, 0x4E2D, 0x1F600};
    if (h % 100 == 0) return wide[(h >> 8) % 7];
    return 'a' + (uint32_t)((h >> 16) % 26);
}
}  // namespace

// Config 5: parent of item i is i-1 with probability p_chain_pct/100, else uniform over
// [0, i-1]; deleted ~ Bernoulli(del_pct/100); cp = 'a' + h % 26; lamport = i; agent = i % 64.
// Counter-based (mix64(seed, i)), so a device generator can reproduce it item by item.
void synth_tree_item(uint64_t seed, uint32_t i, uint32_t p_chain_pct, uint32_t del_pct,
                     uint32_t& par, uint8_t& del, uint32_t& c) {
    uint64_t h0 = mix64(seed, i);
    uint64_t h1 = mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL, i);
    uint64_t h2 = mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL, i);
    par = (h0 % 100 < p_chain_pct) ? i - 1 : (uint32_t)(h1 % i);
    del = (uint8_t)((h2 % 100) < del_pct);
    c = 'a' + (uint32_t)((h2 >> 32) % 26);
}

uint64_t synth_tree_visible(uint32_t n, uint32_t del_pct, uint64_t seed) {
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<uint64_t> part(nt, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            uint64_t c = 0;
            for (uint64_t i = 1 + t; i <= n; i += nt)
                c += (mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL, i) % 100) >= del_pct;
            part[t] = c;
        });
    for (auto& x : th) x.join();
    uint64_t v = 0;
    for (uint64_t c : part) v += c;
    return v;
}

OpLog* synth_tree(uint32_t n, uint32_t p_chain_pct, uint32_t del_pct, uint64_t seed) {
    OpLog* L = new OpLog();
    L->parent.resize(n); L->oright.assign(n, NIL); L->lamport.resize(n);
    L->agent.resize(n); L->deleted.resize(n); L->cp.resize(n);
    uint64_t vis = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        uint32_t par, c;
        uint8_t del;
        synth_tree_item(seed, i, p_chain_pct, del_pct, par, del, c);
        L->parent[i - 1] = par;
        L->lamport[i - 1] = i;
        L->agent[i - 1] = (uint16_t)(i % 64);
        L->deleted[i - 1] = del;
        L->cp[i - 1] = c;
        vis += !del;
    }
    L->max_lamport = n;
    L->mark_stale();  // positional index is rebuilt lazily on a later positional edit
    L->reset_visible(vis);
    return L;
}

// Config 4: `agents` concurrent agents editing in synchronous rounds.  Per round every agent
// performs 1 + Geometric(mean 3) actions against the snapshot taken at round start: a delete
// (20 %) of a random item among the 1,024 most recent visible ones, or an insert run of
// Geometric(mean 8) chars whose first char is anchored (origin_left) at a Zipf(s = 1.2) rank
// over those 1,024 most recent visible items (rank 0 = newest; the document start when the
// snapshot is empty); later chars chain onto the previous one.  All agents of a round share
// the lamport base, so concurrent siblings tie on lamport and are ordered by agent.
OpLog* synth_agents(uint32_t n_items, uint32_t agents, uint64_t seed) {
    OpLog* L = new OpLog();
    if (agents == 0) agents = 1;
    if (agents > 65535) agents = 65535;
    uint64_t st = seed;
    auto rnd = [&] { return splitmix64(st); };
    auto unif = [&] { return (double)(rnd() >> 11) * (1.0 / 9007199254740992.0); };
    auto geom = [&](double mean) {  // >= 1, mean `mean`
        double p = 1.0 / mean;
        double u = unif();
        uint32_t k = 1 + (uint32_t)std::floor(std::log1p(-u) / std::log1p(-p));
        return std::min<uint32_t>(k, 1024);
    };
    const int W = 1024;
    std::vector<double> cdf(W);
    {
        double acc = 0;
        for (int r = 0; r < W; ++r) { acc += 1.0 / std::pow((double)(r + 1), 1.2); cdf[r] = acc; }
        for (double& x : cdf) x /= acc;
    }
    std::vector<uint32_t> created;  // all ids in creation order
    std::vector<uint32_t> snap;     // most recent visible at round start, newest first
    uint32_t base = 0;
    uint32_t n = 0;
    std::vector<uint32_t> pending_dels;
    while (n < n_items) {
        snap.clear();
        for (size_t k = created.size(); k > 0 && snap.size() < (size_t)W; --k) {
            uint32_t id = created[k - 1];
            if (!L->deleted[id - 1]) snap.push_back(id);
        }
        uint32_t round_max = 0;
        pending_dels.clear();
        for (uint32_t a = 0; a < agents && n < n_items; ++a) {
            uint32_t seq = 0;
            uint32_t actions = geom(3.0);
            for (uint32_t act = 0; act < actions && n < n_items; ++act) {
                if (!snap.empty() && unif() < 0.2) {
                    pending_dels.push_back(snap[rnd() % snap.size()]);
                    continue;
                }
                uint32_t anchor = 0;
                if (!snap.empty()) {
                    double u = unif();
                    int r = (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
                    if (r >= (int)snap.size()) r = (int)(rnd() % snap.size());
                    anchor = snap[r];
                }
                uint32_t len = geom(8.0);
                uint32_t prev = anchor;
                for (uint32_t j = 0; j < len && n < n_items; ++j) {
                    ++n;
                    ++seq;
                    L->parent.push_back(prev);
                    L->oright.push_back(NIL);
                    L->lamport.push_back(base + seq);
                    L->agent.push_back((uint16_t)a);
                    L->deleted.push_back(0);
                    L->cp.push_back(pick_cp(rnd()));
                    created.push_back(n);
                    prev = n;
                }
            }
            round_max = std::max(round_max, seq);
        }
        for (uint32_t id : pending_dels) {
            if (!L->deleted[id - 1]) { L->deleted[id - 1] = 1; L->del_ops.push_back(id); }
        }
        base += round_max + 1;
    }
    uint64_t vis = 0;
    for (uint8_t d : L->deleted) vis += !d;
    L->max_lamport = base;
    L->mark_stale();
    L->reset_visible(vis);
    return L;
}

}  // namespace crdt

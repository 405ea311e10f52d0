// bench_main.cpp — C++ restatement of the reference's bench harness (/root/reference/src/main.rs)
// with the GPU engine registered as the CRDT under test, plus the batched group SURVEY.md §8(b)
// proposes.  Accounting as criterion's Throughput::Elements(trace.len()) = patches
// (main.rs:25,58).  Usage: crdt_bench [upstream|downstream|batched|all] [--traces-dir D]
//                          [--iters N] [--replicas R]
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "crdt_hip.h"
#include "hipmerge.hpp"

using hipmerge::check;
using hipmerge::HipMerge;

static const char* TRACES[] = {"automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"};  // main.rs:10-15

struct Loaded {
    crdt_hip_trace* t = nullptr;
    std::string start, end;
    size_t len = 0;
};

static Loaded load(const std::string& dir, const char* name, bool byte_offsets) {
    Loaded L;
    std::string path = dir + "/" + name + ".json.gz";  // main.rs:19
    check(crdt_hip_trace_load(path.c_str(), &L.t), nullptr, "trace_load");
    if (byte_offsets) check(crdt_hip_trace_chars_to_bytes(L.t), nullptr, "chars_to_bytes");  // :21-23
    const char* s;
    size_t n;
    crdt_hip_trace_start_content(L.t, &s, &n);
    L.start.assign(s, n);
    crdt_hip_trace_end_content(L.t, &s, &n);
    L.end.assign(s, n);
    L.len = crdt_hip_trace_len(L.t);
    return L;
}

static void report(const char* group, const char* trace, const char* name, size_t elements,
                   const std::vector<double>& secs) {
    double best = secs[0], sum = 0;
    for (double x : secs) { best = std::min(best, x); sum += x; }
    double mean = sum / secs.size();
    std::printf("%s/%s/%s  time: mean %.3f ms  best %.3f ms  thrpt: %.2f Melem/s (%zu elements, %zu iters)\n",
                group, trace, name, mean * 1e3, best * 1e3, elements / mean / 1e6, elements, secs.size());
    std::fflush(stdout);
}

template <class F>
static std::vector<double> time_iters(int iters, F&& f) {
    std::vector<double> out;
    f();  // warm-up
    for (int i = 0; i < iters; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        f();
        auto t1 = std::chrono::steady_clock::now();
        out.push_back(std::chrono::duration<double>(t1 - t0).count());
    }
    return out;
}

static bool g_fugue = false;  // --order fugue: Fugue logs (left/right anchors, in-order)

// main.rs:17-48 with R = HipMerge
template <class R>
static void upstream(const std::string& dir, const char* name, int iters) {
    Loaded L = load(dir, name, R::EDITS_USE_BYTE_OFFSETS);
    auto secs = time_iters(iters, [&] {
        R rope = R::from_str(L.start, g_fugue);
        for (size_t i = 0; i < L.len; ++i) {
            size_t pos, del, il;
            const char* ins;
            crdt_hip_trace_patch(L.t, i, &pos, &del, &ins, &il);
            rope.replace(pos, pos + del, std::string_view(ins, il));
        }
        size_t got = rope.len();
        if (got != L.end.size()) {  // main.rs:35
            std::fprintf(stderr, "upstream %s: len %zu != %zu\n", name, got, L.end.size());
            std::abort();
        }
    });
    report("upstream", name, R::NAME, L.len, secs);
    crdt_hip_trace_free(L.t);
}

// main.rs:50-81 with R = HipMerge
template <class R>
static void downstream(const std::string& dir, const char* name, int iters) {
    Loaded L = load(dir, name, R::EDITS_USE_BYTE_OFFSETS);
    auto pr = R::upstream_updates(L.start, L.len, [&](size_t i, size_t& pos, size_t& del, std::string_view& ins) {
        const char* p;
        size_t il;
        crdt_hip_trace_patch(L.t, i, &pos, &del, &p, &il);
        ins = std::string_view(p, il);
    }, g_fugue);
    const R& crdt0 = pr.first;
    const auto& updates = pr.second;
    auto secs = time_iters(iters, [&] {
        R crdt = crdt0.clone();                         // main.rs:64
        for (const auto& u : updates) crdt.apply_update(u);  // :65-67
        size_t got = crdt.len();
        if (got != L.end.size()) {                       // :68
            std::fprintf(stderr, "downstream %s: len %zu != %zu\n", name, got, L.end.size());
            std::abort();
        }
    });
    report("downstream", name, R::NAME, L.len, secs);
    crdt_hip_trace_free(L.t);
}

// fn batched(c) — every trace x R replicas resident in HBM, one merge per iter.
static void batched(const std::string& dir, int iters, uint32_t replicas, uint32_t relabel) {
    auto dev = hipmerge::Device::shared();
    std::vector<crdt_hip_oplog*> logs;
    std::vector<crdt_hip_oplog_view> views;
    std::vector<uint64_t> expect_digest;
    size_t patches = 0;
    for (const char* name : TRACES) {
        Loaded L = load(dir, name, false);
        crdt_hip_oplog* log = nullptr;
        check(g_fugue ? crdt_hip_trace_resolve_fugue(L.t, &log) : crdt_hip_trace_resolve(L.t, &log),
              nullptr, "resolve");
        crdt_hip_oplog_view v;
        crdt_hip_oplog_get_view(log, &v);
        logs.push_back(log);
        views.push_back(v);
        expect_digest.push_back(crdt_hip_tree_digest(reinterpret_cast<const uint8_t*>(L.end.data()), L.end.size()));
        patches += L.len;
        crdt_hip_trace_free(L.t);
    }
    crdt_hip_batch* b = nullptr;
    check(crdt_hip_batch_create(dev->ctx, views.data(), (uint32_t)views.size(), replicas, relabel, 1, &b),
          dev->ctx, "batch_create");
    uint64_t docs = 0, items = 0, bytes = 0;
    crdt_hip_batch_info(b, &docs, &items, &bytes);
    std::vector<uint64_t> dig(docs), lens(docs);
    crdt_hip_stats st;
    auto secs = time_iters(iters, [&] {
        check(crdt_hip_batch_merge(dev->ctx, b, dig.data(), lens.data(), &st), dev->ctx, "batch_merge");
    });
    for (uint64_t d = 0; d < docs; ++d)
        if (dig[d] != expect_digest[d % views.size()]) {
            std::fprintf(stderr, "batched: digest mismatch on document %llu\n", (unsigned long long)d);
            std::abort();
        }
    report("batched", "all-4-traces", HipMerge::NAME, patches * replicas, secs);
    std::printf("  docs %llu items %llu device time %.3f ms, all digests match endContent\n",
                (unsigned long long)docs, (unsigned long long)items, st.total_ns / 1e6);
    crdt_hip_batch_free(b);
    for (auto* l : logs) crdt_hip_oplog_free(l);
}

int main(int argc, char** argv) {
    std::string group = argc > 1 ? argv[1] : "all";
    std::string dir = "./traces";  // paths are relative to the CWD, as in main.rs:19
    int iters = 10;
    uint32_t replicas = 64, relabel = 1;
    for (int i = 2; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--traces-dir")) dir = argv[i + 1];
        else if (!std::strcmp(argv[i], "--iters")) iters = std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--replicas")) replicas = (uint32_t)std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--relabel")) relabel = (uint32_t)std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--order")) g_fugue = !std::strcmp(argv[i + 1], "fugue");
    }
    if (group == "upstream" || group == "all")
        for (const char* t : TRACES) upstream<HipMerge>(dir, t, iters);
    if (group == "downstream" || group == "all")
        for (const char* t : TRACES) {
            downstream<HipMerge>(dir, t, iters);       // host decode, device merge
            downstream<hipmerge::HipDownstream>(dir, t, iters);  // device decode + merge
        }
    if (group == "batched" || group == "all") batched(dir, iters, replicas, relabel);
    return 0;
}

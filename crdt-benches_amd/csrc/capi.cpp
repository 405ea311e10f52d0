// capi.cpp — the extern "C" boundary declared in include/crdt_hip.h.  Nothing throws across it:
// every entry point catches, records the message and returns a CRDT_HIP_E* code.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <exception>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "crdt_hip.h"
#include "engine.hpp"
#include "oplog.hpp"
#include "replica.hpp"
#include "store.hpp"
#include "synth.hpp"
#include "trace.hpp"
#include "util.hpp"

struct crdt_hip_ctx {
    crdt::Engine eng;
    std::string last_err;
    crdt::DeviceLogs staging;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
    // replay sessions (crdt_hip_replica_replay): the work replica and learnt sizes per
    // (initial replica, update batch), most recent first
    std::vector<std::unique_ptr<crdt::ReplayState>> replays;
};
struct crdt_hip_oplog {
    crdt::OpLog log;
};
struct crdt_hip_trace {
    crdt::Trace t;
};
struct crdt_hip_batch {
    crdt_hip_ctx* ctx = nullptr;
    crdt::DeviceLogs logs;
    uint64_t device_bytes = 0;
};
struct crdt_hip_replica {
    crdt_hip_ctx* ctx = nullptr;
    crdt::Replica r;
};

struct crdt_hip_updates {
    crdt_hip_ctx* ctx = nullptr;
    crdt::UpdateBatch u;
};

namespace {

// device bytes per op-log slot: parent (4) + key (lamport << 16 | agent, 8) + codepoint (3)
constexpr uint64_t kSlotBytes = 15;
thread_local std::string g_err;

int set_err(crdt_hip_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->last_err = msg;
    else g_err = msg;
    return code;
}
int from_engine(crdt_hip_ctx* ctx, int rc) {
    if (rc) ctx->last_err = ctx->eng.err;
    return rc;
}

template <class F>
int guard(crdt_hip_ctx* ctx, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_err(ctx, CRDT_HIP_ENOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return set_err(ctx, CRDT_HIP_EINVAL, e.what());
    } catch (...) {
        return set_err(ctx, CRDT_HIP_EINVAL, "unknown exception");
    }
}

uint64_t visible_bytes(const crdt_hip_oplog_view& v) {
    // (branch-free, so that it vectorises: part of every crdt_hip_merge of a host view)
    uint64_t b = 0;
    for (uint32_t i = 0; i < v.n; ++i) {
        const uint32_t c = v.cp[i] & 0x1FFFFFu;
        const uint32_t len = 1u + (c >= 0x80u) + (c >= 0x800u) + (c >= 0x10000u);
        b += v.deleted[i] ? 0u : len;
    }
    return b;
}

int check_view(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* v) {
    if (!v) return set_err(ctx, CRDT_HIP_EINVAL, "null op log view");
    if (v->n && (!v->parent || !v->lamport || !v->agent || !v->deleted || !v->cp))
        return set_err(ctx, CRDT_HIP_EINVAL, "op log view has null arrays");
    if (v->n > 0x7FFFFF00u) return set_err(ctx, CRDT_HIP_ERANGE, "op log too large");
    return 0;
}

int stage_views(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* logs, uint32_t n) {
    std::vector<crdt::DocInfo> docs(n);
    for (uint32_t i = 0; i < n; ++i) {
        int rc = check_view(ctx, &logs[i]);
        if (rc) return rc;
        docs[i] = crdt::DocInfo{logs[i].n, visible_bytes(logs[i])};
    }
    int rc = ctx->eng.plan(ctx->staging, docs);
    if (rc) return from_engine(ctx, rc);
    return from_engine(ctx, ctx->eng.upload(ctx->staging, logs, n));
}
}  // namespace

extern "C" {

int crdt_hip_abi_version(void) { return CRDT_HIP_ABI_VERSION; }

int crdt_hip_device_count(int* out) {
    if (!out) return set_err(nullptr, CRDT_HIP_EINVAL, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *out = e == hipSuccess ? n : 0;
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return set_err(nullptr, CRDT_HIP_EDEVICE, hipGetErrorString(e));
    }
    return 0;
}

int crdt_hip_init(int device, crdt_hip_ctx** out) {
    if (!out) return set_err(nullptr, CRDT_HIP_EINVAL, "null out");
    *out = nullptr;
    return guard(nullptr, [&] {
        crdt_hip_ctx* c = new crdt_hip_ctx();
        std::string e = c->eng.init(device);
        if (!e.empty()) {
            delete c;
            return set_err(nullptr, CRDT_HIP_EDEVICE, e);
        }
        *out = c;
        return 0;
    });
}

int crdt_hip_destroy(crdt_hip_ctx* ctx) {
    if (!ctx) return 0;
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    delete ctx;
    return 0;
}

const char* crdt_hip_last_error(const crdt_hip_ctx* ctx) {
    return ctx ? ctx->last_err.c_str() : g_err.c_str();
}

int crdt_hip_set_param(crdt_hip_ctx* ctx, const char* key, uint64_t value) {
    if (!ctx || !key) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    std::string k = key;
    if (k == "splitter_stride") {
        if (value < 16 || value > 4096 || (value & (value - 1)))
            return set_err(ctx, CRDT_HIP_EINVAL, "splitter_stride must be a power of two in [16, 4096]");
        uint32_t l = 0;
        while ((1ull << l) < value) ++l;
        ctx->eng.log2m = l;
        ctx->eng.log2m_set = true;
        return 0;
    }
    if (k == "max_wave_slots") {
        if (value < 4096 || value > (1ull << 31))
            return set_err(ctx, CRDT_HIP_EINVAL, "max_wave_slots out of range");
        ctx->eng.max_wave_slots = value;
        return 0;
    }
    if (k == "tail_wave_div") {
        if (value > 64) return set_err(ctx, CRDT_HIP_EINVAL, "tail_wave_div must be in [0, 64]");
        ctx->eng.tail_wave_div = (uint32_t)value;
        return 0;
    }
    if (k == "lanes") {
        if (value < 1 || value > 8) return set_err(ctx, CRDT_HIP_EINVAL, "lanes must be in [1, 8]");
        ctx->eng.lanes = (uint32_t)value;
        return 0;
    }
    if (k == "lane_gate") {
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "lane_gate must be 0 or 1");
        ctx->eng.l0_gated = value == 1;
        return 0;
    }
    if (k == "l1_split") {
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "l1_split must be 0 or 1");
        ctx->eng.l1_split = value == 1;
        return 0;
    }
    if (k == "plan_cache") {
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "plan_cache must be 0 or 1");
        ctx->eng.plan_cache = value == 1;
        return 0;
    }
    if (k == "fuse_text") {  // 0: k_doctree leaves the text to k_expand (smaller LDS footprint)
        ctx->eng.fuse_text = value != 0;
        return 0;
    }
    if (k == "doctree_lds_max") {  // experiment hook (see Engine::doctree_lds_max)
        ctx->eng.doctree_lds_max = value != 0;
        return 0;
    }
    if (k == "xcd_order") {  // 1: XCD-aware tile order in level 0 (engine.hip xcd_block)
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "xcd_order must be 0 or 1");
        ctx->eng.xcd_order = value == 1;
        return 0;
    }
    if (k == "group_docs") {  // replica batches: documents placed base by base (waves per base)
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "group_docs must be 0 or 1");
        ctx->eng.group_docs = value == 1;
        return CRDT_HIP_OK;
    }
    if (k == "runs_slots") {  // k_runs slots per thread: 16, 32 or 64
        if (value != 16 && value != 32 && value != 64)
            return set_err(ctx, CRDT_HIP_EINVAL, "runs_slots must be 16, 32 or 64");
        ctx->eng.runs_slots = (uint32_t)value;
        return CRDT_HIP_OK;
    }
    if (k == "stile_text") {  // fused plans stage text from the tile segments (L1Plan): 1 by
                              // loads and shifts, 2 by LDS-DMA per tile
        if (value > 2) return set_err(ctx, CRDT_HIP_EINVAL, "stile_text must be 0, 1 or 2");
        ctx->eng.stile_text = (uint32_t)value;
        return 0;
    }
    if (k == "text_scatter") {  // stile plans: 1 k_doctree + k_tscatter, 0 k_doctree phase C
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "text_scatter must be 0 or 1");
        ctx->eng.text_scatter = (uint32_t)value;
        return CRDT_HIP_OK;
    }
    if (k == "contraction") {  // run contraction: 0 by the input, 1 always, 2 never (Wave::nocon)
        if (value > 2) return set_err(ctx, CRDT_HIP_EINVAL, "contraction must be 0, 1 or 2");
        ctx->eng.contraction = (uint32_t)value;
        return CRDT_HIP_OK;
    }
    if (k == "l1_group") {  // global level-1 sibling grouping: 0 auto, 1 counting, 2 radix sorts
        if (value > 2) return set_err(ctx, CRDT_HIP_EINVAL, "l1_group must be 0, 1 or 2");
        ctx->eng.l1_group = (uint32_t)value;
        return CRDT_HIP_OK;
    }
    if (k == "rs_digit_bits") {  // radix sort A's digit width: 0 auto, 8 or 10
        if (value != 0 && value != 8 && value != 10)
            return set_err(ctx, CRDT_HIP_EINVAL, "rs_digit_bits must be 0, 8 or 10");
        ctx->eng.rs_digit_bits = (uint32_t)value;
        return CRDT_HIP_OK;
    }
    if (k == "nsq_list") {  // the compact nsq parent list (Engine::build_nsq, nsq_launch)
        if (value > 2) return set_err(ctx, CRDT_HIP_EINVAL, "nsq_list must be 0, 1 or 2");
        ctx->eng.nsq_list = (uint32_t)value;
        return 0;
    }
    if (k == "doctree_k32") {  // LDS level 1 with 32-bit sibling keys (Engine::doctree_k32)
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "doctree_k32 must be 0 or 1");
        ctx->eng.doctree_k32 = value == 1;
        return CRDT_HIP_OK;
    }
    if (k == "glds_late") {  // test hook (see Engine::glds_late)
        ctx->eng.glds_late = value != 0;
        return 0;
    }
    if (k == "plan_shrink") {  // test hook (see Engine::plan_shrink)
        ctx->eng.plan_shrink = value != 0;
        return 0;
    }
    if (k == "level1") {
        if (value > 1) return set_err(ctx, CRDT_HIP_EINVAL, "level1 must be 0 (auto) or 1 (global)");
        ctx->eng.level1_global = value == 1;
        return 0;
    }
    return set_err(ctx, CRDT_HIP_EINVAL, "unknown parameter " + k);
}

// ---- op log ----------------------------------------------------------------------------------
int crdt_hip_oplog_new(crdt_hip_oplog** out) {
    if (!out) return set_err(nullptr, CRDT_HIP_EINVAL, "null out");
    return guard(nullptr, [&] { *out = new crdt_hip_oplog(); return 0; });
}
int crdt_hip_oplog_set_fugue(crdt_hip_oplog* log, int on) {
    if (!log) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    if (log->log.size()) return set_err(nullptr, CRDT_HIP_EINVAL, "set_fugue needs an empty log");
    log->log.fugue = on != 0;
    return 0;
}
int crdt_hip_oplog_set_agent(crdt_hip_oplog* log, uint16_t agent) {
    if (!log) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    log->log.local_agent = agent;
    return 0;
}
int crdt_hip_oplog_clone(const crdt_hip_oplog* src, crdt_hip_oplog** out) {
    if (!src || !out) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] { *out = new crdt_hip_oplog(*src); return 0; });
}
void crdt_hip_oplog_free(crdt_hip_oplog* log) { delete log; }

int crdt_hip_oplog_insert(crdt_hip_oplog* log, size_t pos, const char* utf8, size_t nbytes) {
    if (!log || (!utf8 && nbytes)) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = log->log.insert_utf8(pos, utf8, nbytes);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_ERANGE, e);
    });
}
int crdt_hip_oplog_remove(crdt_hip_oplog* log, size_t start, size_t end) {
    if (!log) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = log->log.remove(start, end);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_ERANGE, e);
    });
}
int crdt_hip_oplog_replace(crdt_hip_oplog* log, size_t start, size_t end, const char* utf8,
                           size_t nbytes) {
    if (end > start) {
        int rc = crdt_hip_oplog_remove(log, start, end);
        if (rc) return rc;
    }
    if (nbytes) return crdt_hip_oplog_insert(log, start, utf8, nbytes);
    return 0;
}
size_t crdt_hip_oplog_visible_len(const crdt_hip_oplog* log) { return log ? log->log.visible() : 0; }

int crdt_hip_oplog_get_view(const crdt_hip_oplog* log, crdt_hip_oplog_view* out) {
    if (!log || !out) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    const crdt::OpLog& L = log->log;
    out->n = L.size();
    out->parent = L.parent.data();
    out->origin_right = L.oright.data();
    out->lamport = L.lamport.data();
    out->agent = L.agent.data();
    out->deleted = L.deleted.data();
    out->cp = L.cp.data();
    // (non-NULL for an empty Fugue log too: a replica made from it is a Fugue replica)
    static const uint8_t kNoSide = 0;
    out->side = L.fugue ? (L.side.empty() ? &kNoSide : L.side.data()) : nullptr;
    return 0;
}
uint64_t crdt_hip_oplog_version(const crdt_hip_oplog* log) { return log ? log->log.version() : 0; }

int crdt_hip_oplog_encode_from(const crdt_hip_oplog* log, uint64_t version, uint8_t* buf,
                               size_t cap, size_t* out_len) {
    if (!log || !out_len) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::vector<uint8_t> u = log->log.encode_from(version);
        *out_len = u.size();
        if (!buf || cap < u.size()) return set_err(nullptr, CRDT_HIP_ESPACE, "buffer too small");
        std::memcpy(buf, u.data(), u.size());
        return 0;
    });
}
int crdt_hip_oplog_apply_update(crdt_hip_oplog* log, const uint8_t* buf, size_t len) {
    if (!log || (!buf && len)) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = log->log.apply_update(buf, len);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_EINVAL, e);
    });
}

// ---- traces ----------------------------------------------------------------------------------
int crdt_hip_trace_load(const char* path, crdt_hip_trace** out) {
    if (!path || !out) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    *out = nullptr;
    return guard(nullptr, [&] {
        crdt_hip_trace* t = new crdt_hip_trace();
        std::string e = crdt::load_trace(path, t->t);
        if (!e.empty()) {
            delete t;
            return set_err(nullptr, CRDT_HIP_EIO, e);
        }
        *out = t;
        return 0;
    });
}
void crdt_hip_trace_free(crdt_hip_trace* t) { delete t; }
size_t crdt_hip_trace_len(const crdt_hip_trace* t) { return t ? t->t.len() : 0; }
size_t crdt_hip_trace_txns(const crdt_hip_trace* t) { return t ? t->t.txn_end.size() : 0; }

int crdt_hip_trace_patch(const crdt_hip_trace* t, size_t i, size_t* pos, size_t* del,
                         const char** ins, size_t* ins_len) {
    if (!t || i >= t->t.patches.size()) return set_err(nullptr, CRDT_HIP_ERANGE, "patch index");
    const crdt::Patch& p = t->t.patches[i];
    if (pos) *pos = p.pos;
    if (del) *del = p.del;
    if (ins) *ins = t->t.ins.data() + p.ins_off;
    if (ins_len) *ins_len = p.ins_len;
    return 0;
}
int crdt_hip_trace_start_content(const crdt_hip_trace* t, const char** s, size_t* len) {
    if (!t || !s || !len) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    *s = t->t.start_content.data();
    *len = t->t.start_content.size();
    return 0;
}
int crdt_hip_trace_end_content(const crdt_hip_trace* t, const char** s, size_t* len) {
    if (!t || !s || !len) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    *s = t->t.end_content.data();
    *len = t->t.end_content.size();
    return 0;
}
int crdt_hip_trace_chars_to_bytes(crdt_hip_trace* t) {
    if (!t) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = crdt::chars_to_bytes(t->t);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_ERANGE, e);
    });
}
namespace {
int trace_resolve(const crdt_hip_trace* t, crdt_hip_oplog** out, bool fugue);
}
int crdt_hip_trace_resolve(const crdt_hip_trace* t, crdt_hip_oplog** out) {
    return trace_resolve(t, out, false);
}
int crdt_hip_trace_resolve_fugue(const crdt_hip_trace* t, crdt_hip_oplog** out) {
    return trace_resolve(t, out, true);
}
namespace {
int trace_resolve(const crdt_hip_trace* t, crdt_hip_oplog** out, bool fugue) {
    if (!t || !out) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    if (t->t.byte_offsets)
        return set_err(nullptr, CRDT_HIP_EINVAL, "resolve needs codepoint offsets (EDITS_USE_BYTE_OFFSETS = false)");
    *out = nullptr;
    return guard(nullptr, [&] {
        crdt_hip_oplog* L = new crdt_hip_oplog();
        L->log.fugue = fugue;
        const crdt::Trace& T = t->t;
        std::string e;
        // (OpLog::replay sizes the columns to the patches' bounds itself)
        // from_str(start_content), then replace() every patch (main.rs:29-33, rope.rs:21-32)
        if (!T.start_content.empty())
            e = L->log.insert_utf8(0, T.start_content.data(), T.start_content.size());
        static_assert(sizeof(crdt::Patch) == 4 * sizeof(uint64_t), "Patch = {pos, del, ins_off, ins_len}");
        if (e.empty())
            e = L->log.replay(reinterpret_cast<const uint64_t*>(T.patches.data()), T.patches.size(),
                              T.ins.data(), T.ins.size());
        if (!e.empty()) {
            delete L;
            return set_err(nullptr, CRDT_HIP_ERANGE, e);
        }
        *out = L;
        return 0;
    });
}
}  // namespace

int crdt_hip_trace_resolve_many(const crdt_hip_trace* const* traces, uint32_t n, uint32_t threads,
                                crdt_hip_oplog** out) {
    if ((n && (!traces || !out))) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i) {
        out[i] = nullptr;
        if (!traces[i]) return set_err(nullptr, CRDT_HIP_EINVAL, "null trace");
    }
    uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    uint32_t k = threads ? threads : std::min(n, hw);
    k = std::max(1u, std::min(k, n ? n : 1u));
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    std::atomic<uint32_t> next{0};
    auto work = [&] {
        for (uint32_t i; (i = next.fetch_add(1)) < n;) {
            rc[i] = crdt_hip_trace_resolve(traces[i], &out[i]);
            if (rc[i]) msg[i] = crdt_hip_last_error(nullptr);  // (thread-local: read it here)
        }
    };
    std::vector<std::thread> pool;
    try {
        pool.reserve(k);
        for (uint32_t j = 1; j < k; ++j) pool.emplace_back(work);
    } catch (...) {
        // no more threads (std::system_error) or no memory: the threads already started and
        // the calling thread share the work; nothing may cross the C ABI
    }
    work();
    for (std::thread& th : pool) th.join();
    for (uint32_t i = 0; i < n; ++i)
        if (rc[i]) {
            for (uint32_t j = 0; j < n; ++j) {
                if (out[j]) crdt_hip_oplog_free(out[j]);
                out[j] = nullptr;
            }
            return set_err(nullptr, rc[i], "trace " + std::to_string(i) + ": " + msg[i]);
        }
    return 0;
}

// ---- binary files ----------------------------------------------------------------------------
struct crdt_hip_logfile {
    crdt::MappedLog m;
};

int crdt_hip_trace_save(const crdt_hip_trace* t, const char* path) {
    if (!t || !path) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = crdt::save_trace_bin(t->t, path);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_EIO, e);
    });
}
int crdt_hip_oplog_save(const crdt_hip_oplog* log, const char* path) {
    if (!log || !path) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    return guard(nullptr, [&] {
        std::string e = crdt::save_oplog(log->log, path);
        return e.empty() ? 0 : set_err(nullptr, CRDT_HIP_EIO, e);
    });
}
int crdt_hip_oplog_load(const char* path, crdt_hip_oplog** out) {
    if (!path || !out) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    *out = nullptr;
    return guard(nullptr, [&] {
        crdt_hip_oplog* L = new crdt_hip_oplog();
        std::string e = crdt::load_oplog(path, L->log);
        if (!e.empty()) {
            delete L;
            return set_err(nullptr, CRDT_HIP_EIO, e);
        }
        *out = L;
        return 0;
    });
}
int crdt_hip_logfile_open(const char* path, crdt_hip_logfile** out, crdt_hip_oplog_view* view) {
    if (!path || !out || !view) return set_err(nullptr, CRDT_HIP_EINVAL, "null argument");
    *out = nullptr;
    return guard(nullptr, [&] {
        crdt_hip_logfile* f = new crdt_hip_logfile();
        std::string e = crdt::map_oplog(path, f->m);
        if (!e.empty()) {
            delete f;
            return set_err(nullptr, CRDT_HIP_EIO, e);
        }
        view->n = f->m.n;
        view->parent = f->m.parent;
        view->origin_right = f->m.oright;
        view->lamport = f->m.lamport;
        view->agent = f->m.agent;
        view->deleted = f->m.deleted;
        view->cp = f->m.cp;
        static const uint8_t kNoSide = 0;  // (an empty Fugue file's view is still Fugue)
        view->side = f->m.fugue ? (f->m.n ? f->m.side : &kNoSide) : nullptr;
        *out = f;
        return 0;
    });
}
int crdt_hip_logfile_close(crdt_hip_logfile* f) {
    delete f;
    return 0;
}

// ---- synthetic -------------------------------------------------------------------------------
int crdt_hip_synth_agents(uint32_t n_items, uint32_t agents, uint64_t seed, crdt_hip_oplog** out) {
    if (!out) return set_err(nullptr, CRDT_HIP_EINVAL, "null out");
    return guard(nullptr, [&] {
        crdt::OpLog* L = crdt::synth_agents(n_items, agents, seed);
        crdt_hip_oplog* o = new crdt_hip_oplog();
        o->log = std::move(*L);
        delete L;
        *out = o;
        return 0;
    });
}
int crdt_hip_synth_tree_visible(uint32_t n_items, uint32_t del_pct, uint64_t seed, uint64_t* out) {
    if (!out || del_pct > 100) return set_err(nullptr, CRDT_HIP_EINVAL, "bad arguments");
    return guard(nullptr, [&] { *out = crdt::synth_tree_visible(n_items, del_pct, seed); return 0; });
}
int crdt_hip_synth_tree(uint32_t n_items, uint32_t p_chain_pct, uint32_t del_pct, uint64_t seed,
                        crdt_hip_oplog** out) {
    if (!out) return set_err(nullptr, CRDT_HIP_EINVAL, "null out");
    if (p_chain_pct > 100 || del_pct > 100) return set_err(nullptr, CRDT_HIP_EINVAL, "percent > 100");
    return guard(nullptr, [&] {
        crdt::OpLog* L = crdt::synth_tree(n_items, p_chain_pct, del_pct, seed);
        crdt_hip_oplog* o = new crdt_hip_oplog();
        o->log = std::move(*L);
        delete L;
        *out = o;
        return 0;
    });
}

// ---- merge -----------------------------------------------------------------------------------
int crdt_hip_merge(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint8_t* out, size_t cap,
                   size_t* out_len, uint64_t* digest) {
    if (!ctx) return set_err(nullptr, CRDT_HIP_EINVAL, "null context");
    return guard(ctx, [&] {
        int rc = stage_views(ctx, log, 1);
        if (rc) return rc;
        std::vector<uint8_t> text;
        std::vector<uint64_t> offs;
        uint64_t dig = 0, len = 0;
        rc = ctx->eng.merge(ctx->staging, crdt::Engine::TEXT, &dig, &len, nullptr,
                            out ? &text : nullptr, nullptr);
        if (rc) return from_engine(ctx, rc);
        if (out_len) *out_len = (size_t)len;
        if (digest) *digest = dig;
        if (out) {
            if (cap < len) return set_err(ctx, CRDT_HIP_ESPACE, "output buffer too small");
            if (len) std::memcpy(out, text.data(), (size_t)len);
        }
        return 0;
    });
}

int crdt_hip_merge_len(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint64_t* codepoints,
                       uint64_t* bytes, uint64_t* digest) {
    if (!ctx) return set_err(nullptr, CRDT_HIP_EINVAL, "null context");
    return guard(ctx, [&] {
        int rc = stage_views(ctx, log, 1);
        if (rc) return rc;
        uint64_t dig = 0, len = 0, cps = 0;
        rc = ctx->eng.merge(ctx->staging, crdt::Engine::TEXT, &dig, &len, nullptr, nullptr,
                            nullptr, &cps);
        if (rc) return from_engine(ctx, rc);
        if (codepoints) *codepoints = cps;
        if (bytes) *bytes = len;
        if (digest) *digest = dig;
        return 0;
    });
}

int crdt_hip_merge_batch(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* logs, uint32_t n,
                         uint64_t* digests, uint64_t* lens, crdt_hip_stats* stats) {
    if (!ctx || (!logs && n)) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    return guard(ctx, [&] {
        if (n == 0) return 0;
        int rc = stage_views(ctx, logs, n);
        if (rc) return rc;
        return from_engine(ctx, ctx->eng.merge(ctx->staging, crdt::Engine::TEXT, digests, lens, stats));
    });
}

int crdt_hip_merge_order(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* log, uint32_t* order) {
    if (!ctx || !order) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    return guard(ctx, [&] {
        int rc = stage_views(ctx, log, 1);
        if (rc) return rc;
        std::vector<uint8_t> raw;
        rc = ctx->eng.merge(ctx->staging, crdt::Engine::ORDER, nullptr, nullptr, nullptr, &raw, nullptr);
        if (rc) return from_engine(ctx, rc);
        if (raw.size() != (size_t)log->n * 4)
            return set_err(ctx, CRDT_HIP_EBADLOG, "order output size mismatch");
        if (!raw.empty()) std::memcpy(order, raw.data(), raw.size());
        return 0;
    });
}

// ---- resident batches ------------------------------------------------------------------------
int crdt_hip_batch_create(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* bases, uint32_t nbases,
                          uint32_t replicas, uint32_t relabel, uint64_t seed,
                          crdt_hip_batch** out) {
    if (!ctx || !bases || !out || nbases == 0 || replicas == 0)
        return set_err(ctx, CRDT_HIP_EINVAL, "bad batch arguments");
    if (relabel > 2) return set_err(ctx, CRDT_HIP_EINVAL, "relabel must be 0, 1 or 2");
    *out = nullptr;
    return guard(ctx, [&] {
        int rc = stage_views(ctx, bases, nbases);
        if (rc) return rc;
        crdt_hip_batch* b = new crdt_hip_batch();
        b->ctx = ctx;
        rc = ctx->eng.replicate(ctx->staging, b->logs, replicas, relabel, seed);
        if (rc) {
            delete b;
            return from_engine(ctx, rc);
        }
        b->device_bytes = b->logs.total_slots * kSlotBytes + (b->logs.total_slots >> b->logs.log2m) * 4;
        *out = b;
        return 0;
    });
}
int crdt_hip_batch_synth_tree(crdt_hip_ctx* ctx, uint32_t n_items, uint32_t p_chain_pct,
                              uint32_t del_pct, uint64_t seed, crdt_hip_batch** out) {
    if (!ctx || !out || p_chain_pct > 100 || del_pct > 100)
        return set_err(ctx, CRDT_HIP_EINVAL, "bad synth arguments");
    *out = nullptr;
    return guard(ctx, [&] {
        crdt_hip_batch* b = new crdt_hip_batch();
        b->ctx = ctx;
        int rc = ctx->eng.synth_tree(b->logs, n_items, p_chain_pct, del_pct, seed);
        if (rc) {
            delete b;
            return from_engine(ctx, rc);
        }
        b->device_bytes = b->logs.total_slots * kSlotBytes + (b->logs.total_slots >> b->logs.log2m) * 4;
        *out = b;
        return 0;
    });
}
int crdt_hip_batch_free(crdt_hip_batch* b) {
    delete b;
    return 0;
}
int crdt_hip_batch_info(const crdt_hip_batch* b, uint64_t* docs, uint64_t* items,
                        uint64_t* device_bytes) {
    if (!b) return set_err(nullptr, CRDT_HIP_EINVAL, "null batch");
    if (docs) *docs = b->logs.docs.size();
    if (items) *items = b->logs.items;
    if (device_bytes) *device_bytes = b->device_bytes;
    return 0;
}
int crdt_hip_batch_merge(crdt_hip_ctx* ctx, crdt_hip_batch* b, uint64_t* digests, uint64_t* lens,
                         crdt_hip_stats* stats) {
    if (!ctx || !b) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (b->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "batch belongs to another context");
    return guard(ctx, [&] {
        return from_engine(ctx, ctx->eng.merge(b->logs, crdt::Engine::TEXT, digests, lens, stats));
    });
}

int crdt_hip_batch_raw(crdt_hip_ctx* ctx, crdt_hip_batch* b, int on) {
    if (!ctx || !b) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (b->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "batch belongs to another context");
    return guard(ctx, [&] {
        if (!on) {
            b->logs.raw = false;
            return 0;
        }
        if (b->logs.raw_lam) {
            b->logs.raw = true;
            return 0;
        }
        return from_engine(ctx, ctx->eng.raw_keep(b->logs));
    });
}

// ---- device-resident replicas ----------------------------------------------------------------
int crdt_hip_replica_new(crdt_hip_ctx* ctx, const crdt_hip_oplog_view* init,
                         crdt_hip_replica** out) {
    if (!ctx || !out) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    *out = nullptr;
    if (init) {
        int rc = check_view(ctx, init);
        if (rc) return rc;
    }
    return guard(ctx, [&] {
        crdt_hip_replica* r = new crdt_hip_replica();
        r->ctx = ctx;
        int rc = crdt::replica_upload(ctx->eng, r->r, init);
        if (rc) {
            delete r;
            return from_engine(ctx, rc);
        }
        *out = r;
        return 0;
    });
}
int crdt_hip_replica_clone(crdt_hip_ctx* ctx, const crdt_hip_replica* src,
                           crdt_hip_replica** out) {
    if (!ctx || !src || !out) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (src->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "replica belongs to another context");
    *out = nullptr;
    return guard(ctx, [&] {
        crdt_hip_replica* r = new crdt_hip_replica();
        r->ctx = ctx;
        int rc = crdt::replica_copy(ctx->eng, src->r, r->r);
        if (rc) {
            delete r;
            return from_engine(ctx, rc);
        }
        *out = r;
        return 0;
    });
}
namespace {
void drop_replays(crdt_hip_ctx* ctx, const void* init, const void* ub) {
    if (!ctx) return;
    auto& v = ctx->replays;
    for (size_t i = v.size(); i-- > 0;)
        if (v[i]->init == init || v[i]->ub == ub) v.erase(v.begin() + (long)i);
}
}  // namespace

int crdt_hip_replica_free(crdt_hip_replica* r) {
    if (r) drop_replays(r->ctx, &r->r, nullptr);
    delete r;
    return 0;
}
int crdt_hip_replica_apply_updates(crdt_hip_ctx* ctx, crdt_hip_replica* r, const uint8_t* buf,
                                   size_t len, const uint64_t* offsets, uint32_t n) {
    if (!ctx || !r) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (r->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "replica belongs to another context");
    return guard(ctx, [&] {
        return from_engine(ctx, crdt::replica_apply(ctx->eng, r->r, buf, len, offsets, n));
    });
}
int crdt_hip_updates_upload(crdt_hip_ctx* ctx, const uint8_t* buf, size_t len,
                            const uint64_t* offsets, uint32_t n, crdt_hip_updates** out) {
    if (!ctx || !out) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    return guard(ctx, [&] {
        crdt_hip_updates* u = new crdt_hip_updates();
        u->ctx = ctx;
        int rc = crdt::updates_upload(ctx->eng, u->u, buf, len, offsets, n);
        if (rc) {
            delete u;
            return from_engine(ctx, rc);
        }
        *out = u;
        return 0;
    });
}
int crdt_hip_updates_free(crdt_hip_updates* u) {
    if (u) drop_replays(u->ctx, nullptr, &u->u);
    delete u;
    return 0;
}

int crdt_hip_replica_replay(crdt_hip_ctx* ctx, const crdt_hip_replica* init,
                            const crdt_hip_updates* u, uint64_t* codepoints, uint64_t* bytes,
                            uint64_t* digest) {
    if (!ctx || !init || !u) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (init->ctx != ctx || u->ctx != ctx)
        return set_err(ctx, CRDT_HIP_EINVAL, "replica or updates belong to another context");
    return guard(ctx, [&] {
        auto& v = ctx->replays;
        size_t i = 0;
        while (i < v.size() && !(v[i]->init == &init->r && v[i]->ub == &u->u)) ++i;
        if (i == v.size()) {
            if (v.size() >= 8) v.pop_back();
            v.insert(v.begin(), std::make_unique<crdt::ReplayState>());
            i = 0;
        }
        uint64_t c = 0, b = 0, d = 0;
        const int rc = crdt::replica_replay(ctx->eng, init->r, u->u, *v[i], &c, &b, &d);
        if (rc) return from_engine(ctx, rc);
        if (codepoints) *codepoints = c;
        if (bytes) *bytes = b;
        if (digest) *digest = d;
        return 0;
    });
}
int crdt_hip_replica_apply_resident(crdt_hip_ctx* ctx, crdt_hip_replica* r,
                                    const crdt_hip_updates* u) {
    if (!ctx || !r || !u) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (r->ctx != ctx || u->ctx != ctx)
        return set_err(ctx, CRDT_HIP_EINVAL, "replica or updates belong to another context");
    return guard(ctx, [&] {
        return from_engine(ctx, crdt::replica_apply_resident(ctx->eng, r->r, u->u));
    });
}
int crdt_hip_replica_info(const crdt_hip_replica* r, uint64_t* items,
                          uint64_t* visible_codepoints, uint64_t* visible_bytes) {
    if (!r) return set_err(nullptr, CRDT_HIP_EINVAL, "null replica");
    if (items) *items = r->r.n;
    if (visible_codepoints) *visible_codepoints = r->r.vis_cp;
    if (visible_bytes) *visible_bytes = r->r.vis_bytes;
    return 0;
}
int crdt_hip_replica_merge(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint8_t* out, size_t cap,
                           size_t* out_len, uint64_t* digest) {
    if (!ctx || !r) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (r->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "replica belongs to another context");
    return guard(ctx, [&] {
        std::vector<uint8_t> text;
        uint64_t len = 0, dig = 0;
        int rc = crdt::replica_merge(ctx->eng, r->r, out ? &text : nullptr, &len, &dig, nullptr);
        if (rc) return from_engine(ctx, rc);
        if (out_len) *out_len = (size_t)len;
        if (digest) *digest = dig;
        if (out) {
            if (cap < len) return set_err(ctx, CRDT_HIP_ESPACE, "output buffer too small");
            if (len) std::memcpy(out, text.data(), (size_t)len);
        }
        return 0;
    });
}

int crdt_hip_replica_merge_len(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint64_t* codepoints,
                               uint64_t* bytes, uint64_t* digest) {
    if (!ctx || !r) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (r->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "replica belongs to another context");
    return guard(ctx, [&] {
        uint64_t len = 0, dig = 0, cps = 0;
        int rc = crdt::replica_merge(ctx->eng, r->r, nullptr, &len, &dig, nullptr, &cps);
        if (rc) return from_engine(ctx, rc);
        if (codepoints) *codepoints = cps;
        if (bytes) *bytes = len;
        if (digest) *digest = dig;
        return 0;
    });
}

int crdt_hip_replica_merge_inc(crdt_hip_ctx* ctx, crdt_hip_replica* r, uint8_t* out, size_t cap,
                               size_t* out_len, uint64_t* codepoints, uint32_t* path) {
    if (!ctx || !r) return set_err(ctx, CRDT_HIP_EINVAL, "null argument");
    if (r->ctx != ctx) return set_err(ctx, CRDT_HIP_EINVAL, "replica belongs to another context");
    return guard(ctx, [&] {
        std::vector<uint8_t> text;
        uint64_t len = 0, cps = 0;
        uint32_t p = 0;
        int rc = crdt::replica_merge_inc(ctx->eng, r->r, out ? &text : nullptr, &len, &cps, &p);
        if (rc) return from_engine(ctx, rc);
        if (out_len) *out_len = (size_t)len;
        if (codepoints) *codepoints = cps;
        if (path) *path = p;
        if (out) {
            if (cap < len) return set_err(ctx, CRDT_HIP_ESPACE, "output buffer too small");
            if (len) std::memcpy(out, text.data(), (size_t)len);
        }
        return 0;
    });
}

// ---- RCCL ------------------------------------------------------------------------------------
int crdt_hip_comm_unique_id(uint8_t id[128]) {
    if (!id) return set_err(nullptr, CRDT_HIP_EINVAL, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return set_err(nullptr, CRDT_HIP_ECOMM, ncclGetErrorString(r));
    std::memcpy(id, &u, 128);
    return 0;
}
int crdt_hip_comm_init(crdt_hip_ctx* ctx, int nranks, int rank, const uint8_t id[128]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return set_err(ctx, CRDT_HIP_EINVAL, "bad comm arguments");
    if (hipSetDevice(ctx->eng.device) != hipSuccess)
        return set_err(ctx, CRDT_HIP_EDEVICE, "hipSetDevice failed");
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) return set_err(ctx, CRDT_HIP_ECOMM, ncclGetErrorString(r));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return 0;
}
int crdt_hip_allgather_u64(crdt_hip_ctx* ctx, const uint64_t* send, size_t count, uint64_t* recv) {
    if (!ctx || !ctx->comm || (!send && count) || (!recv && count))
        return set_err(ctx, CRDT_HIP_EINVAL, "comm not initialised or null buffer");
    if (count == 0) return 0;
    uint64_t *ds = nullptr, *dr = nullptr;
    hipStream_t s = ctx->eng.stream;
    auto cleanup = [&] {
        if (ds) (void)hipFree(ds);
        if (dr) (void)hipFree(dr);
    };
    if (hipMalloc(&ds, count * 8) != hipSuccess ||
        hipMalloc(&dr, count * 8 * (size_t)ctx->nranks) != hipSuccess) {
        cleanup();
        return set_err(ctx, CRDT_HIP_ENOMEM, "device allocation for all-gather");
    }
    hipError_t e = hipMemcpyAsync(ds, send, count * 8, hipMemcpyHostToDevice, s);
    ncclResult_t r = ncclSuccess;
    if (e == hipSuccess) r = ncclAllGather(ds, dr, count, ncclUint64, ctx->comm, s);
    if (e == hipSuccess && r == ncclSuccess)
        e = hipMemcpyAsync(recv, dr, count * 8 * (size_t)ctx->nranks, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    cleanup();
    if (r != ncclSuccess) return set_err(ctx, CRDT_HIP_ECOMM, ncclGetErrorString(r));
    if (e != hipSuccess) return set_err(ctx, CRDT_HIP_EDEVICE, hipGetErrorString(e));
    return 0;
}
int crdt_hip_comm_destroy(crdt_hip_ctx* ctx) {
    if (!ctx) return 0;
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    return 0;
}

// ---- helpers ---------------------------------------------------------------------------------
uint64_t crdt_hip_xxh64(const void* data, size_t len, uint64_t seed) { return crdt::xxh64(data, len, seed); }
uint64_t crdt_hip_tree_digest(const uint8_t* text, size_t len) { return crdt::tree_digest(text, len); }

}  // extern "C"

// store.cpp — trace cache and op-log files (store.hpp).  Layouts, little-endian:
//
// trace cache: magic "CRDTTRC1", u32 version, u32 flags (bit 0: byte offsets), u64 patches,
//   u64 txns, u64 inserted bytes, u64 start bytes, u64 end bytes; then patches as
//   {u64 pos, u64 del, u64 ins_off, u64 ins_len}, u32 txn_end[txns], start, end, inserted text.
//
// op-log file: magic "CRDTLOG1", u32 version, u32 n, u32 delete ops, u16 local agent, u16 0,
//   u32 max lamport, u64 file size, u64 offset[7] of parent, origin_right, lamport, cp (u32 each),
//   agent (u16), deleted (u8), delete-op targets (u32); every array starts on a 64-byte boundary.
#include "store.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <vector>

namespace crdt {

namespace {

struct LogHeader {
    char magic[8];
    uint32_t version, n, ndels;
    uint16_t local_agent, pad;
    uint32_t max_lamport;
    uint64_t size;
    uint64_t off[7];
};
static_assert(sizeof(LogHeader) == 96, "op-log header layout");

struct TraceHeader {
    char magic[8];
    uint32_t version, flags;
    uint64_t npatches, ntxns, nins, nstart, nend;
};
static_assert(sizeof(TraceHeader) == 56, "trace header layout");

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
};

std::string write_all(const std::string& path, const std::vector<std::pair<const void*, size_t>>& parts) {
    const std::string tmp = path + ".tmp";
    File w;
    w.f = std::fopen(tmp.c_str(), "wb");
    if (!w.f) return "cannot create " + tmp;
    for (const auto& p : parts)
        if (p.second && std::fwrite(p.first, 1, p.second, w.f) != p.second) return "write error on " + tmp;
    if (std::fclose(w.f) != 0) {
        w.f = nullptr;
        return "write error on " + tmp;
    }
    w.f = nullptr;
    if (std::rename(tmp.c_str(), path.c_str()) != 0) return "cannot rename " + tmp;
    return "";
}

std::string read_all(const std::string& path, std::vector<uint8_t>& out) {
    File r;
    r.f = std::fopen(path.c_str(), "rb");
    if (!r.f) return "cannot open " + path;
    if (std::fseek(r.f, 0, SEEK_END) != 0) return "cannot seek " + path;
    const long sz = std::ftell(r.f);
    if (sz < 0) return "cannot size " + path;
    std::fseek(r.f, 0, SEEK_SET);
    out.resize((size_t)sz);
    if (sz && std::fread(out.data(), 1, (size_t)sz, r.f) != (size_t)sz) return "read error on " + path;
    return "";
}

uint64_t align64(uint64_t x) { return (x + 63u) & ~63ull; }

}  // namespace

bool is_trace_bin(const std::string& path) {
    File r;
    r.f = std::fopen(path.c_str(), "rb");
    char m[8];
    return r.f && std::fread(m, 1, 8, r.f) == 8 && std::memcmp(m, kTraceMagic, 8) == 0;
}

std::string save_trace_bin(const Trace& t, const std::string& path) {
    TraceHeader h{};
    std::memcpy(h.magic, kTraceMagic, 8);
    h.version = kStoreVersion;
    h.flags = t.byte_offsets ? 1u : 0u;
    h.npatches = t.patches.size();
    h.ntxns = t.txn_end.size();
    h.nins = t.ins.size();
    h.nstart = t.start_content.size();
    h.nend = t.end_content.size();
    static_assert(sizeof(Patch) == 32, "patch layout");
    return write_all(path, {{&h, sizeof h},
                            {t.patches.data(), t.patches.size() * sizeof(Patch)},
                            {t.txn_end.data(), t.txn_end.size() * 4},
                            {t.start_content.data(), t.start_content.size()},
                            {t.end_content.data(), t.end_content.size()},
                            {t.ins.data(), t.ins.size()}});
}

std::string load_trace_bin(const std::string& path, Trace& out) {
    std::vector<uint8_t> b;
    std::string e = read_all(path, b);
    if (!e.empty()) return e;
    TraceHeader h;
    if (b.size() < sizeof h) return "truncated trace cache " + path;
    std::memcpy(&h, b.data(), sizeof h);
    if (std::memcmp(h.magic, kTraceMagic, 8) != 0) return "not a trace cache: " + path;
    if (h.version != kStoreVersion) return "unsupported trace cache version in " + path;
    const uint64_t lim = b.size();
    if (h.npatches > lim / sizeof(Patch) || h.ntxns > lim / 4 || h.nins > lim || h.nstart > lim ||
        h.nend > lim)
        return "corrupt trace cache " + path;
    const uint64_t need = sizeof h + h.npatches * sizeof(Patch) + h.ntxns * 4 + h.nstart + h.nend + h.nins;
    if (need != b.size()) return "truncated trace cache " + path;
    const uint8_t* p = b.data() + sizeof h;
    Trace t;
    t.byte_offsets = (h.flags & 1u) != 0;
    t.patches.resize(h.npatches);
    std::memcpy(t.patches.data(), p, h.npatches * sizeof(Patch));
    p += h.npatches * sizeof(Patch);
    t.txn_end.resize(h.ntxns);
    std::memcpy(t.txn_end.data(), p, h.ntxns * 4);
    p += h.ntxns * 4;
    t.start_content.assign(reinterpret_cast<const char*>(p), h.nstart);
    p += h.nstart;
    t.end_content.assign(reinterpret_cast<const char*>(p), h.nend);
    p += h.nend;
    t.ins.assign(reinterpret_cast<const char*>(p), h.nins);
    for (const Patch& q : t.patches)
        if (q.ins_off > h.nins || q.ins_len > h.nins - q.ins_off) return "corrupt trace cache " + path;
    uint32_t prev = 0;
    for (uint32_t x : t.txn_end) {
        if (x < prev || x > h.npatches) return "corrupt trace cache " + path;
        prev = x;
    }
    out = std::move(t);
    return "";
}

std::string save_oplog(const OpLog& L, const std::string& path) {
    LogHeader h{};
    std::memcpy(h.magic, kLogMagic, 8);
    h.version = L.fugue ? kLogVersionFugue : kStoreVersion;
    h.n = L.size();
    h.ndels = (uint32_t)L.del_ops.size();
    if (L.fugue && L.side.size() != L.size()) return "malformed Fugue op log (side column)";
    h.local_agent = L.local_agent;
    h.max_lamport = L.max_lamport;
    const uint64_t n = h.n;
    const uint64_t bytes[7] = {4 * n, 4 * n, 4 * n, 4 * n, 2 * n, n, 4ull * h.ndels};
    const void* src[7] = {L.parent.data(), L.oright.data(), L.lamport.data(), L.cp.data(),
                          L.agent.data(), L.deleted.data(), L.del_ops.data()};
    uint64_t at = align64(sizeof h);
    for (int i = 0; i < 7; ++i) {
        h.off[i] = at;
        at = align64(at + bytes[i]);
    }
    const uint64_t side_off = at;  // (Fugue) the side column follows the arrays
    if (L.fugue) at = align64(at + n);
    h.size = at;
    static const uint8_t zeros[64] = {};
    std::vector<std::pair<const void*, size_t>> parts{{&h, sizeof h}};
    uint64_t pos = sizeof h;
    for (int i = 0; i < 7; ++i) {
        parts.push_back({zeros, (size_t)(h.off[i] - pos)});
        parts.push_back({src[i], (size_t)bytes[i]});
        pos = h.off[i] + bytes[i];
    }
    if (L.fugue) {
        parts.push_back({zeros, (size_t)(side_off - pos)});
        parts.push_back({L.side.data(), (size_t)n});
        pos = side_off + n;
    }
    parts.push_back({zeros, (size_t)(h.size - pos)});
    return write_all(path, parts);
}

MappedLog::~MappedLog() {
    if (base) munmap(base, size);
}

std::string map_oplog(const std::string& path, MappedLog& out) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return "cannot open " + path;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return "cannot stat " + path;
    }
    const size_t size = (size_t)st.st_size;
    if (size < sizeof(LogHeader)) {
        close(fd);
        return "truncated op-log file " + path;
    }
    void* base = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (base == MAP_FAILED) return "cannot map " + path;
    LogHeader h;
    std::memcpy(&h, base, sizeof h);
    auto fail = [&](const char* what) {
        munmap(base, size);
        return std::string(what) + path;
    };
    if (std::memcmp(h.magic, kLogMagic, 8) != 0) return fail("not an op-log file: ");
    if (h.version != kStoreVersion && h.version != kLogVersionFugue)
        return fail("unsupported op-log file version in ");
    if (h.size != size) return fail("truncated op-log file ");
    const uint64_t n = h.n;
    const uint64_t bytes[7] = {4 * n, 4 * n, 4 * n, 4 * n, 2 * n, n, 4ull * h.ndels};
    for (int i = 0; i < 7; ++i)
        if (h.off[i] % 64 || h.off[i] < sizeof h || h.off[i] > size || bytes[i] > size - h.off[i])
            return fail("corrupt op-log file ");
    const bool fugue = h.version == kLogVersionFugue;
    const uint64_t side_off = align64(h.off[6] + bytes[6]);
    if (fugue && (side_off > size || n > size - side_off)) return fail("corrupt op-log file ");
    const uint8_t* b = static_cast<const uint8_t*>(base);
    if (out.base) munmap(out.base, out.size);
    out.base = base;
    out.size = size;
    out.n = h.n;
    out.ndels = h.ndels;
    out.local_agent = h.local_agent;
    out.max_lamport = h.max_lamport;
    out.parent = reinterpret_cast<const uint32_t*>(b + h.off[0]);
    out.oright = reinterpret_cast<const uint32_t*>(b + h.off[1]);
    out.lamport = reinterpret_cast<const uint32_t*>(b + h.off[2]);
    out.cp = reinterpret_cast<const uint32_t*>(b + h.off[3]);
    out.agent = reinterpret_cast<const uint16_t*>(b + h.off[4]);
    out.deleted = b + h.off[5];
    out.del_ops = reinterpret_cast<const uint32_t*>(b + h.off[6]);
    out.fugue = fugue;
    out.side = fugue ? b + side_off : nullptr;
    return "";
}

std::string load_oplog(const std::string& path, OpLog& out) {
    MappedLog m;
    std::string e = map_oplog(path, m);
    if (!e.empty()) return e;
    OpLog L;
    L.local_agent = m.local_agent;
    L.parent.assign(m.parent, m.parent + m.n);
    L.oright.assign(m.oright, m.oright + m.n);
    L.lamport.assign(m.lamport, m.lamport + m.n);
    L.cp.assign(m.cp, m.cp + m.n);
    L.agent.assign(m.agent, m.agent + m.n);
    L.deleted.assign(m.deleted, m.deleted + m.n);
    L.del_ops.assign(m.del_ops, m.del_ops + m.ndels);
    if (m.fugue) {
        L.fugue = true;
        L.side.assign(m.side, m.side + m.n);
    }
    uint64_t vis = 0;
    uint32_t ml = 0;
    for (uint32_t i = 0; i < m.n; ++i) {
        vis += !L.deleted[i];
        if (L.lamport[i] > ml) ml = L.lamport[i];
    }
    L.max_lamport = std::max(ml, m.max_lamport);
    L.reset_visible(vis);
    L.mark_stale();
    out = std::move(L);
    return "";
}

}  // namespace crdt

// store.hpp — binary files for the two inputs of the merge path:
//   * a trace cache: the parsed josephg trace (patches, inserted text, start/end content) in one
//     flat little-endian file, so that a run skips gunzip + JSON (load_testing_data,
//     /root/reference/src/main.rs:19,52);
//   * an op-log file: the resolved anchor op log as 64-byte-aligned SoA arrays, mapped read-only
//     so that its arrays are a crdt_hip_oplog_view without a copy (a merge, a batch_create or a
//     replica upload reads them straight from the page cache).
#pragma once
#include <cstdint>
#include <string>

#include "oplog.hpp"
#include "trace.hpp"

namespace crdt {

constexpr char kTraceMagic[8] = {'C', 'R', 'D', 'T', 'T', 'R', 'C', '1'};
constexpr char kLogMagic[8] = {'C', 'R', 'D', 'T', 'L', 'O', 'G', '1'};
constexpr uint32_t kStoreVersion = 1;
// Op-log files of Fugue logs: version 2, the same header and arrays followed by the side column
// (n bytes, 64-byte aligned).  Readers take both versions.
constexpr uint32_t kLogVersionFugue = 2;

bool is_trace_bin(const std::string& path);
std::string save_trace_bin(const Trace& t, const std::string& path);
std::string load_trace_bin(const std::string& path, Trace& out);

std::string save_oplog(const OpLog& L, const std::string& path);

// A read-only mapping of an op-log file.  Arrays point into the mapping.
struct MappedLog {
    void* base = nullptr;
    size_t size = 0;
    uint32_t n = 0, ndels = 0;
    uint16_t local_agent = 0;
    uint32_t max_lamport = 0;
    const uint32_t *parent = nullptr, *oright = nullptr, *lamport = nullptr, *cp = nullptr;
    const uint16_t* agent = nullptr;
    const uint8_t* deleted = nullptr;
    const uint32_t* del_ops = nullptr;
    const uint8_t* side = nullptr;  // Fugue files (version 2); NULL otherwise
    bool fugue = false;
    ~MappedLog();
};
std::string map_oplog(const std::string& path, MappedLog& out);
// An editable op log from a file (the positional index is rebuilt on the first edit).
std::string load_oplog(const std::string& path, OpLog& out);

}  // namespace crdt

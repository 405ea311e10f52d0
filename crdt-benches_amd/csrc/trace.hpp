// trace.hpp — josephg editing-trace loader.  Restates crdt-testdata's load_testing_data /
// TestData::{len, chars_to_bytes} (used at /root/reference/src/main.rs:19-25,52-58):
// gzip + JSON {startContent, endContent, txns: [{time, patches: [[pos, del, ins], ...]}]}.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace crdt {

struct Patch {
    uint64_t pos;      // codepoints (or bytes after chars_to_bytes)
    uint64_t del;      // codepoints (or bytes)
    uint64_t ins_off;  // byte offset of the inserted UTF-8 in Trace::ins
    uint64_t ins_len;  // bytes
};

struct Trace {
    std::string start_content, end_content;
    std::vector<Patch> patches;          // all txns flattened, in replay order (main.rs:30-31)
    std::vector<uint32_t> txn_end;       // patches index one past each txn
    std::string ins;                     // concatenated inserted text
    bool byte_offsets = false;

    size_t len() const { return patches.size(); }  // TestData::len == number of patches
};

// Returns "" on success, else an error message.
std::string load_trace(const std::string& path, Trace& out);
std::string parse_trace_json(const char* data, size_t n, Trace& out);
// TestData::chars_to_bytes: rewrite (pos, del) from codepoints to UTF-8 bytes.
std::string chars_to_bytes(Trace& t);

}  // namespace crdt

// hipmerge.hpp — C++ mirror of the reference's per-CRDT adapter interface for the GPU engine,
// written against the C ABI only (include/crdt_hip.h), exactly as the Rust `impl Upstream /
// Downstream for HipMerge` in INTEGRATION.md is.
//
//   trait Upstream   /root/reference/src/rope.rs:6-33
//   trait Downstream /root/reference/src/rope.rs:185-191
//   Dt adapter it sits beside: /root/reference/src/rope.rs:105-137, :193-225
#pragma once
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "crdt_hip.h"

namespace hipmerge {

// Panic on error, matching the harness's unwrap/assert style (rope.rs:53, main.rs:35).
inline void check(int rc, const crdt_hip_ctx* ctx, const char* what) {
    if (rc != CRDT_HIP_OK) {
        std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, crdt_hip_last_error(ctx));
        std::abort();
    }
}

// One device context shared by every clone (clones never copy device buffers).
struct Device {
    crdt_hip_ctx* ctx = nullptr;
    explicit Device(int dev) { check(crdt_hip_init(dev, &ctx), nullptr, "crdt_hip_init"); }
    ~Device() { crdt_hip_destroy(ctx); }
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    // The process-wide device, never destroyed: a static destructor would run crdt_hip_destroy
    // after the HIP runtime's own teardown at exit (the process exit releases the device).
    static std::shared_ptr<Device> shared() {
        static std::shared_ptr<Device>* d = new std::shared_ptr<Device>(std::make_shared<Device>(0));
        return *d;
    }
};

class HipMerge {
public:
    static constexpr const char* NAME = "mi355x";
    static constexpr bool EDITS_USE_BYTE_OFFSETS = false;
    using Update = std::vector<uint8_t>;

    // Upstream::from_str (rope.rs:113-121: new op log, one insert of the start content);
    // `fugue`: a Fugue log (left/right anchors, in-order document, version-2 updates)
    static HipMerge from_str(std::string_view s, bool fugue = false) {
        HipMerge m;
        if (fugue) check(crdt_hip_oplog_set_fugue(m.log_.get(), 1), nullptr, "set_fugue");
        if (!s.empty()) m.insert(0, s);
        return m;
    }
    void insert(size_t at, std::string_view s) {
        check(crdt_hip_oplog_insert(log_.get(), at, s.data(), s.size()), nullptr, "insert");
    }
    void remove(size_t start, size_t end) {
        check(crdt_hip_oplog_remove(log_.get(), start, end), nullptr, "remove");
    }
    // Upstream::replace default (rope.rs:21-32)
    void replace(size_t start, size_t end, std::string_view s) {
        if (end > start) remove(start, end);
        if (!s.empty()) insert(start, s);
    }
    // Upstream::len: the merge (Dt: checkout_tip().len(), rope.rs:134-136).  Codepoints.
    size_t len() const {
        crdt_hip_oplog_view v;
        check(crdt_hip_oplog_get_view(log_.get(), &v), nullptr, "view");
        uint64_t cps = 0;
        check(crdt_hip_merge_len(dev_->ctx, &v, &cps, nullptr, nullptr), dev_->ctx,
              "crdt_hip_merge_len");
        return (size_t)cps;
    }
    std::string text() const {
        crdt_hip_oplog_view v;
        check(crdt_hip_oplog_get_view(log_.get(), &v), nullptr, "view");
        std::string out((size_t)v.n * 4 + 16, '\0');
        size_t n = 0;
        check(crdt_hip_merge(dev_->ctx, &v, reinterpret_cast<uint8_t*>(out.data()), out.size(), &n,
                             nullptr),
              dev_->ctx, "crdt_hip_merge");
        out.resize(n);
        return out;
    }
    uint64_t digest() const {
        crdt_hip_oplog_view v;
        check(crdt_hip_oplog_get_view(log_.get(), &v), nullptr, "view");
        size_t n = 0;
        uint64_t d = 0;
        check(crdt_hip_merge(dev_->ctx, &v, nullptr, 0, &n, &d), dev_->ctx, "crdt_hip_merge");
        return d;
    }
    // Borrowed SoA view of the host op log (valid until the next mutation).
    crdt_hip_oplog_view view() const {
        crdt_hip_oplog_view v;
        check(crdt_hip_oplog_get_view(log_.get(), &v), nullptr, "view");
        return v;
    }
    const std::shared_ptr<Device>& device() const { return dev_; }
    HipMerge clone() const {
        crdt_hip_oplog* c = nullptr;
        check(crdt_hip_oplog_clone(log_.get(), &c), nullptr, "clone");
        return HipMerge(c, dev_);
    }

    // Downstream::upstream_updates (rope.rs:196-220): replay on an upstream copy, encoding one
    // update per patch from the previous version.
    template <class PatchFn>
    static std::pair<HipMerge, std::vector<Update>> upstream_updates(std::string_view start,
                                                                      size_t npatches,
                                                                      PatchFn&& patch,
                                                                      bool fugue = false) {
        HipMerge up = from_str(start, fugue);
        std::vector<Update> updates;
        updates.reserve(npatches);
        for (size_t i = 0; i < npatches; ++i) {
            size_t pos, del;
            std::string_view ins;
            patch(i, pos, del, ins);
            uint64_t v = crdt_hip_oplog_version(up.log_.get());
            up.replace(pos, pos + del, ins);
            size_t need = 0;
            (void)crdt_hip_oplog_encode_from(up.log_.get(), v, nullptr, 0, &need);
            Update u(need);
            check(crdt_hip_oplog_encode_from(up.log_.get(), v, u.data(), u.size(), &need), nullptr,
                  "encode_from");
            updates.push_back(std::move(u));
        }
        return {from_str(start, fugue), std::move(updates)};
    }
    // Downstream::apply_update (rope.rs:222-224)
    void apply_update(const Update& u) {
        check(crdt_hip_oplog_apply_update(log_.get(), u.data(), u.size()), nullptr, "apply_update");
    }

private:
    struct Free {
        void operator()(crdt_hip_oplog* l) const { crdt_hip_oplog_free(l); }
    };
    std::unique_ptr<crdt_hip_oplog, Free> log_;
    std::shared_ptr<Device> dev_;

    HipMerge() : dev_(Device::shared()) {
        crdt_hip_oplog* l = nullptr;
        check(crdt_hip_oplog_new(&l), nullptr, "oplog_new");
        log_.reset(l);
    }
    HipMerge(crdt_hip_oplog* l, std::shared_ptr<Device> d) : log_(l), dev_(std::move(d)) {}
};

// Downstream with the replica resident on the device (crdt_hip_replica_*).  apply_update only
// queues the encoded update in a host buffer; len() decodes every queued update on the device in
// one batch (the decode_and_add of rope.rs:222-224 for all of them), merges the replica where it
// lies and returns its visible codepoints.  clone() copies the replica device to device.
class HipDownstream {
public:
    static constexpr const char* NAME = "mi355x-device";
    static constexpr bool EDITS_USE_BYTE_OFFSETS = false;
    using Update = HipMerge::Update;

    template <class PatchFn>
    static std::pair<HipDownstream, std::vector<Update>> upstream_updates(std::string_view start,
                                                                           size_t npatches,
                                                                           PatchFn&& patch,
                                                                           bool fugue = false) {
        auto pr = HipMerge::upstream_updates(start, npatches, patch, fugue);
        crdt_hip_oplog_view v = pr.first.view();
        HipDownstream d(pr.first.device());
        // (a Fugue log's view, empty or not, makes a Fugue replica)
        check(crdt_hip_replica_new(d.dev_->ctx, v.n || v.side ? &v : nullptr, &d.rep_), d.dev_->ctx,
              "replica_new");
        return {std::move(d), std::move(pr.second)};
    }
    HipDownstream(HipDownstream&& o) noexcept
        : dev_(std::move(o.dev_)), rep_(o.rep_), buf_(std::move(o.buf_)), off_(std::move(o.off_)) {
        o.rep_ = nullptr;
    }
    HipDownstream(const HipDownstream&) = delete;
    ~HipDownstream() {
        if (rep_) crdt_hip_replica_free(rep_);
    }
    HipDownstream clone() const {  // main.rs:64
        HipDownstream c(dev_);
        check(crdt_hip_replica_clone(dev_->ctx, rep_, &c.rep_), dev_->ctx, "replica_clone");
        c.buf_ = buf_;
        c.off_ = off_;
        return c;
    }
    void apply_update(const Update& u) {  // rope.rs:222-224 (queued)
        buf_.insert(buf_.end(), u.begin(), u.end());
        off_.push_back(buf_.size());
    }
    // Upstream::len (codepoints) of the merged document: counted on the device from the merged
    // bytes, cross-checked against the decoder's counters.
    size_t len() const {
        flush();
        uint64_t mcps = 0, mbytes = 0, items = 0, cps = 0, bytes = 0;
        check(crdt_hip_replica_merge_len(dev_->ctx, rep_, &mcps, &mbytes, nullptr), dev_->ctx,
              "replica_merge_len");
        crdt_hip_replica_info(rep_, &items, &cps, &bytes);
        if (mcps != cps || mbytes != bytes) {
            std::fprintf(stderr, "replica: merged %llu codepoints / %llu bytes, decoder %llu / %llu\n",
                         (unsigned long long)mcps, (unsigned long long)mbytes,
                         (unsigned long long)cps, (unsigned long long)bytes);
            std::abort();
        }
        return (size_t)mcps;
    }
    std::string text() const {
        flush();
        uint64_t items = 0, cps = 0, bytes = 0;
        crdt_hip_replica_info(rep_, &items, &cps, &bytes);
        std::string out((size_t)bytes + 16, '\0');
        size_t n = 0;
        check(crdt_hip_replica_merge(dev_->ctx, rep_, reinterpret_cast<uint8_t*>(out.data()),
                                     out.size(), &n, nullptr),
              dev_->ctx, "replica_merge");
        out.resize(n);
        return out;
    }

private:
    std::shared_ptr<Device> dev_;
    crdt_hip_replica* rep_ = nullptr;
    mutable std::vector<uint8_t> buf_;
    mutable std::vector<uint64_t> off_{0};

    explicit HipDownstream(std::shared_ptr<Device> d) : dev_(std::move(d)) {}
    void flush() const {
        if (off_.size() < 2) return;
        check(crdt_hip_replica_apply_updates(dev_->ctx, rep_, buf_.data(), buf_.size(), off_.data(),
                                             (uint32_t)(off_.size() - 1)),
              dev_->ctx, "replica_apply_updates");
        buf_.clear();
        off_.assign(1, 0);
    }
};

}  // namespace hipmerge

/*
 * oracle.h — CPU restatement of the replay-and-merge path of noib3/crdt-benches.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (crdt-benches_amd/, include/) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * Parity pinning: the reference (Rust, crates.io deps, no lockfile) cannot be built or run
 * here.  The oracle is pinned by the reference's own fixtures: the `endContent` string of
 * each trace under traces/ (the same bytes the reference's length assert compares against,
 * /root/reference/src/main.rs:35,68), and by the digests in SURVEY.md §4.2.
 * Multi-agent (concurrent) merge order is "parity unpinned": no reference test or trace
 * exercises concurrency; it is pinned only by two independent oracles below agreeing.
 *
 * Semantics followed:
 *   - replay:   /root/reference/src/main.rs:28-36 (from_str, replay every TestPatch, len)
 *               /root/reference/src/rope.rs:21-32 (replace = remove(start..end) then insert)
 *               /root/reference/src/rope.rs:16-19 (codepoint offsets, EDITS_USE_BYTE_OFFSETS=false)
 *   - resolve:  the positional -> identity step inside diamond-types OpLog::add_insert /
 *               add_delete_without_content (/root/reference/src/rope.rs:116-131), restated with
 *               the RGA anchor conventions of SURVEY.md §4.2.
 *   - merge:    OpLog::checkout_tip (/root/reference/src/rope.rs:135): op log -> document.
 */
#ifndef CRDT_ORACLE_H
#define CRDT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* xxHash64 (Yann Collet's published algorithm, spec v0.8). */
uint64_t orc_xxh64(const void* data, size_t len, uint64_t seed);

/* Tree digest of a document: xxh64 of the little-endian concatenation of the xxh64 (seed 0)
 * of each 4096-byte leaf, seeded with the byte length.  Same definition as the device digest. */
uint64_t orc_tree_digest(const uint8_t* text, size_t len);

/* UTF-8 encode `n` codepoints; returns bytes written (<= 4n). */
size_t orc_utf8_encode(const uint32_t* cp, size_t n, uint8_t* out);

/* Patches: patch i deletes del[i] codepoints at pos[i], then inserts the ins_len[i] codepoints
 * ins_cp[ins_off[i] ..].  start_cp/start_n = startContent. */
typedef struct {
    size_t npatch;
    const uint64_t* pos;
    const uint64_t* del;
    const uint64_t* ins_off;
    const uint64_t* ins_len;
    const uint32_t* ins_cp;
    const uint32_t* start_cp;
    size_t start_n;
} orc_patches;

/* Positional replay into a codepoint gap buffer.  Writes UTF-8 to out (cap bytes).
 * Returns the byte length, or -1 on a bad patch / -2 if cap is too small. */
int64_t orc_replay(const orc_patches* p, uint8_t* out, size_t cap);
/* Same, returning the final codepoint count only (the reference's len()). */
int64_t orc_replay_len(const orc_patches* p);

/* Resolve patches into an anchor op log (ids 1..n, id 0 = document start).
 * Arrays must hold start_n + sum(ins_len) entries.  Returns n, or -1 on a bad patch.
 * lamport[i] = i+1, agent = 0 (single agent "bench", rope.rs:117). */
int64_t orc_resolve(const orc_patches* p, uint32_t* parent, uint32_t* oright,
                    uint32_t* lamport, uint16_t* agent, uint8_t* deleted, uint32_t* cp);

/* RGA merge by tree construction + iterative pre-order DFS: parent = origin_left, siblings
 * ordered by (lamport, agent) descending.  Writes UTF-8 text; optional `order` gets the
 * pre-order item ids (all n items, tombstones included).  Returns byte length, -1 on a
 * malformed log (bad parent / cycle), -2 if cap too small. */
int64_t orc_merge_rga(uint32_t n, const uint32_t* parent, const uint32_t* lamport,
                      const uint16_t* agent, const uint8_t* deleted, const uint32_t* cp,
                      uint8_t* out, size_t cap, uint32_t* order);

/* Fugue mode (Weidner & Kleppmann, "The Art of the Fugue", 2023), the other document order the
 * survey names ("side u8 (Fugue)", "in-order (Fugue)").  Every item is
 * a left (side[i] != 0) or right child of parent[i]; the document is the in-order walk: an
 * item's left children, the item, its right children, siblings on each side by (lamport, agent)
 * descending (ties: greater id first), as in the RGA order.  With no left children this is
 * exactly orc_merge_rga.  Sibling order among concurrent inserts is parity unpinned (diamond-
 * types' FugueMax tie rules are not available); sequential traces pin it through endContent.
 * Same return convention as orc_merge_rga; a left child of the document start is malformed. */
int64_t orc_merge_fugue(uint32_t n, const uint32_t* parent, const uint8_t* side,
                        const uint32_t* lamport, const uint16_t* agent, const uint8_t* deleted,
                        const uint32_t* cp, uint8_t* out, size_t cap, uint32_t* order);

/* Resolver with Fugue anchors: an insert after left neighbour `a` (the p-th visible item, or the
 * start) whose full-list successor is `b` becomes a right child of `a` when `a` has no right
 * child yet, else a left child of `b` (then the leftmost node of a's right subtree).  Same
 * arrays as orc_resolve plus side[]. */
int64_t orc_resolve_fugue(const orc_patches* p, uint32_t* parent, uint8_t* side,
                          uint32_t* lamport, uint16_t* agent, uint8_t* deleted, uint32_t* cp);

/* Independent O(n^2) RGA integrator: items integrated in (lamport, agent) order into a linked
 * list, each after its parent skipping every following item with a greater timestamp.  For
 * small logs (cross-checks the tree oracle).  Same return convention. */
int64_t orc_merge_rga_naive(uint32_t n, const uint32_t* parent, const uint32_t* lamport,
                            const uint16_t* agent, const uint8_t* deleted, const uint32_t* cp,
                            uint8_t* out, size_t cap);

/* Batched CPU merge used as the bench's cpu_baseline: merges `nlogs` logs with `threads`
 * threads, each log independently (same algorithm as orc_merge_rga), storing the tree digest
 * of each result.  Returns 0 or a negative error. */
typedef struct {
    uint32_t n;
    const uint32_t* parent;
    const uint32_t* lamport;
    const uint16_t* agent;
    const uint8_t* deleted;
    const uint32_t* cp;
} orc_log;
int orc_merge_many(const orc_log* logs, uint32_t nlogs, int threads, uint64_t* digests,
                   uint64_t* lens);

#ifdef __cplusplus
}
#endif
#endif

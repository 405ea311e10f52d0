// synth.hpp — synthetic anchor op logs for SURVEY.md §8(d) configs 4 and 5.
#pragma once
#include <cstdint>

namespace crdt {
class OpLog;
void synth_tree_item(uint64_t seed, uint32_t i, uint32_t p_chain_pct, uint32_t del_pct,
                     uint32_t& par, uint8_t& del, uint32_t& c);
OpLog* synth_tree(uint32_t n, uint32_t p_chain_pct, uint32_t del_pct, uint64_t seed);
// Visible (non-deleted) items of synth_tree(n, *, del_pct, seed), without building the log.
uint64_t synth_tree_visible(uint32_t n, uint32_t del_pct, uint64_t seed);
OpLog* synth_agents(uint32_t n_items, uint32_t agents, uint64_t seed);
}  // namespace crdt

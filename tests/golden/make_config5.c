/*
 * make_config5.c — golden digests of SURVEY.md §8(d) config 5 at its full size (1 G items).
 *
 * TEST INFRASTRUCTURE.  Generates the synthetic single-document log of config 5 (splitmix64
 * seed 0x5EED0002: parent of item i = i - 1 with probability p_chain, else uniform over
 * [0, i - 1]; deleted = Bernoulli(del_pct); content 'a' + h % 26; lamport = i; agent = i mod 64)
 * item by item with the same counter-based hashes as the product's generator
 * (crdt-benches_amd/csrc/synth.cpp synth_tree_item, restated here, not linked), merges it with
 * the oracle's sequential RGA merge (oracle/oracle.c orc_merge_rga, the restatement of
 * checkout_tip, /root/reference/src/rope.rs:135) and prints one JSON object with the merged
 * length and the tree digest.  tests/golden/config5.json holds the output for p_chain 90 and 0;
 * tests/test_gpu_scale.py compares the device merge of the same log against it, which pins the
 * ORDER of the 500 M visible items, not only their count (the reference's own check is the
 * length assert, /root/reference/src/main.rs:35,68).
 *
 * Build + run (about 32 GB of memory and a few minutes per case, single-threaded):
 *   make -C oracle && gcc -O2 -o /tmp/make_config5 tests/golden/make_config5.c \
 *       -Loracle -loracle -Wl,-rpath,$PWD/oracle
 *   /tmp/make_config5 1000000000 90 50 && /tmp/make_config5 1000000000 0 50
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../../oracle/oracle.h"

static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint64_t mix64(uint64_t seed, uint64_t i) {
    uint64_t s = seed ^ (i * 0xD1B54A32D192ED03ULL);
    return splitmix64(&s);
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s n p_chain_pct del_pct [seed]\n", argv[0]);
        return 2;
    }
    const uint32_t n = (uint32_t)strtoull(argv[1], 0, 0);
    const uint32_t pc = (uint32_t)atoi(argv[2]), dp = (uint32_t)atoi(argv[3]);
    const uint64_t seed = argc > 4 ? strtoull(argv[4], 0, 0) : 0x5EED0002ull;
    uint32_t* parent = malloc((size_t)n * 4);
    uint32_t* lamport = malloc((size_t)n * 4);
    uint16_t* agent = malloc((size_t)n * 2);
    uint8_t* deleted = malloc((size_t)n);
    uint32_t* cp = malloc((size_t)n * 4);
    if (!parent || !lamport || !agent || !deleted || !cp) return 3;
    uint64_t vis = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        const uint64_t h0 = mix64(seed, i);
        const uint64_t h1 = mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL, i);
        const uint64_t h2 = mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL, i);
        parent[i - 1] = (h0 % 100 < pc) ? i - 1 : (uint32_t)(h1 % i);
        deleted[i - 1] = (uint8_t)((h2 % 100) < dp);
        cp[i - 1] = 'a' + (uint32_t)((h2 >> 32) % 26);
        lamport[i - 1] = i;
        agent[i - 1] = (uint16_t)(i % 64);
        vis += !deleted[i - 1];
    }
    uint8_t* out = malloc(vis + 16);
    const clock_t t0 = clock();
    const int64_t len = orc_merge_rga(n, parent, lamport, agent, deleted, cp, out, vis + 16, NULL);
    const double secs = (double)(clock() - t0) / CLOCKS_PER_SEC;
    if (len < 0) {
        fprintf(stderr, "merge failed: %" PRId64 "\n", len);
        return 1;
    }
    const uint64_t dig = orc_tree_digest(out, (size_t)len);
    printf("{\"n\": %u, \"p_chain\": %u, \"del_pct\": %u, \"seed\": %" PRIu64
           ", \"len\": %" PRId64 ", \"visible\": %" PRIu64 ", \"digest\": \"%016" PRIx64
           "\", \"merge_s\": %.1f}\n",
           n, pc, dp, seed, len, vis, dig, secs);
    return 0;
}

/*
 * oracle.c — CPU restatement of the replay-and-merge path (TEST INFRASTRUCTURE ONLY).
 * See oracle.h for the reference file:line each function follows and how it is pinned.
 * Plain C99, no dependencies beyond libc + pthreads.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* xxHash64 — restated from the published xxHash specification (XXH64).                       */
/* ------------------------------------------------------------------------------------------ */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * XP1 + XP4;
}

uint64_t orc_xxh64(const void* data, size_t len, uint64_t seed) {
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        const uint8_t* lim = end - 32;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xround(0, rd64(p));
        h = rotl64(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * XP5;
        h = rotl64(h, 11) * XP1;
        ++p;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

uint64_t orc_tree_digest(const uint8_t* text, size_t len) {
    const size_t LEAF = 4096;
    size_t nleaf = (len + LEAF - 1) / LEAF;
    uint8_t* buf = (uint8_t*)malloc(nleaf * 8 + 1);
    for (size_t i = 0; i < nleaf; ++i) {
        size_t n = len - i * LEAF < LEAF ? len - i * LEAF : LEAF;
        uint64_t h = orc_xxh64(text + i * LEAF, n, 0);
        for (int b = 0; b < 8; ++b) buf[i * 8 + b] = (uint8_t)(h >> (8 * b));
    }
    /* more than 4096 leaves (16 MiB): the leaf digests are hashed in groups of 4096 (seed =
     * group index) and the document digest is taken over the group digests */
    const size_t GROUP = 4096;
    size_t nd = nleaf;
    if (nleaf > GROUP) {
        size_t ngroup = (nleaf + GROUP - 1) / GROUP;
        for (size_t k = 0; k < ngroup; ++k) {
            size_t n = nleaf - k * GROUP < GROUP ? nleaf - k * GROUP : GROUP;
            uint64_t h = orc_xxh64(buf + k * GROUP * 8, n * 8, (uint64_t)k);
            for (int b = 0; b < 8; ++b) buf[k * 8 + b] = (uint8_t)(h >> (8 * b));
        }
        nd = ngroup;
    }
    uint64_t d = orc_xxh64(buf, nd * 8, (uint64_t)len);
    free(buf);
    return d;
}

/* ------------------------------------------------------------------------------------------ */
/* UTF-8                                                                                       */
/* ------------------------------------------------------------------------------------------ */
static inline size_t enc1(uint32_t c, uint8_t* o) {
    if (c < 0x80) { o[0] = (uint8_t)c; return 1; }
    if (c < 0x800) { o[0] = 0xC0 | (c >> 6); o[1] = 0x80 | (c & 63); return 2; }
    if (c < 0x10000) {
        o[0] = 0xE0 | (c >> 12); o[1] = 0x80 | ((c >> 6) & 63); o[2] = 0x80 | (c & 63);
        return 3;
    }
    o[0] = 0xF0 | (c >> 18); o[1] = 0x80 | ((c >> 12) & 63);
    o[2] = 0x80 | ((c >> 6) & 63); o[3] = 0x80 | (c & 63);
    return 4;
}
static inline size_t len1(uint32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; }

size_t orc_utf8_encode(const uint32_t* cp, size_t n, uint8_t* out) {
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) k += enc1(cp[i], out + k);
    return k;
}

/* ------------------------------------------------------------------------------------------ */
/* Positional replay (src/main.rs:28-36, src/rope.rs:21-32) on a codepoint gap buffer.         */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint32_t* b; size_t cap, gs, ge; } gapbuf; /* gap = [gs, ge) */

static size_t gb_len(const gapbuf* g) { return g->cap - (g->ge - g->gs); }
static void gb_move(gapbuf* g, size_t pos) {
    if (pos < g->gs) {
        size_t n = g->gs - pos;
        memmove(g->b + g->ge - n, g->b + pos, n * 4);
        g->gs -= n; g->ge -= n;
    } else if (pos > g->gs) {
        size_t n = pos - g->gs;
        memmove(g->b + g->gs, g->b + g->ge, n * 4);
        g->gs += n; g->ge += n;
    }
}
static int gb_reserve(gapbuf* g, size_t need) {
    if (g->ge - g->gs >= need) return 0;
    size_t len = gb_len(g);
    size_t ncap = (len + need) * 2 + 64;
    uint32_t* nb = (uint32_t*)malloc(ncap * 4);
    if (!nb) return -1;
    size_t tail = g->cap - g->ge;
    memcpy(nb, g->b, g->gs * 4);
    memcpy(nb + ncap - tail, g->b + g->ge, tail * 4);
    free(g->b);
    g->b = nb; g->ge = ncap - tail; g->cap = ncap;
    return 0;
}

static int replay_into(const orc_patches* p, gapbuf* g) {
    g->b = NULL; g->cap = g->gs = g->ge = 0;
    /* from_str(start_content) == insert(0, s) */
    if (gb_reserve(g, p->start_n + 1)) return -1;
    memcpy(g->b, p->start_cp, p->start_n * 4);
    g->gs += p->start_n;
    for (size_t i = 0; i < p->npatch; ++i) {
        size_t pos = p->pos[i], del = p->del[i];
        size_t len = gb_len(g);
        if (pos > len || del > len - pos) return -1;
        gb_move(g, pos);
        g->ge += del; /* remove(pos..pos+del) */
        size_t il = p->ins_len[i];
        if (il) {
            if (gb_reserve(g, il)) return -1;
            memcpy(g->b + g->gs, p->ins_cp + p->ins_off[i], il * 4);
            g->gs += il;
        }
    }
    return 0;
}

int64_t orc_replay(const orc_patches* p, uint8_t* out, size_t cap) {
    gapbuf g;
    if (replay_into(p, &g)) { free(g.b); return -1; }
    size_t need = 0;
    for (size_t i = 0; i < g.gs; ++i) need += len1(g.b[i]);
    for (size_t i = g.ge; i < g.cap; ++i) need += len1(g.b[i]);
    if (need > cap) { free(g.b); return -2; }
    size_t k = orc_utf8_encode(g.b, g.gs, out);
    k += orc_utf8_encode(g.b + g.ge, g.cap - g.ge, out + k);
    free(g.b);
    return (int64_t)k;
}

int64_t orc_replay_len(const orc_patches* p) {
    gapbuf g;
    if (replay_into(p, &g)) { free(g.b); return -1; }
    int64_t n = (int64_t)gb_len(&g);
    free(g.b);
    return n;
}

/* ------------------------------------------------------------------------------------------ */
/* Resolver: positional patches -> anchor op log (RGA conventions).            */
/* A doubly linked list over all items (tombstones included) with one cached cursor; editing   */
/* traces are local so the cursor walk is short.  Deliberately independent of the product's   */
/* order-statistic resolver.                                                                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t *next, *prev;
    uint8_t* dead;
    uint32_t cur;  /* cursor item */
    uint64_t cnt;  /* visible items in [start .. cur] inclusive */
} rlist;

#define NIL 0xFFFFFFFFu

/* Move the cursor to the p-th visible item (p = 0: the start sentinel, id 0). */
static int rl_seek(rlist* L, uint64_t p) {
    while (L->cnt < p) {
        uint32_t nx = L->next[L->cur];
        if (nx == NIL) return -1;
        L->cur = nx;
        if (!L->dead[nx]) L->cnt++;
    }
    while (L->cnt > p || (L->cur != 0 && L->dead[L->cur])) {
        if (!L->dead[L->cur]) L->cnt--;
        L->cur = L->prev[L->cur];
    }
    return 0;
}

int64_t orc_resolve(const orc_patches* p, uint32_t* parent, uint32_t* oright, uint32_t* lamport,
                    uint16_t* agent, uint8_t* deleted, uint32_t* cp) {
    size_t total = p->start_n;
    for (size_t i = 0; i < p->npatch; ++i) total += p->ins_len[i];
    rlist L;
    L.next = (uint32_t*)malloc((total + 1) * 4);
    L.prev = (uint32_t*)malloc((total + 1) * 4);
    L.dead = (uint8_t*)calloc(total + 1, 1);
    L.next[0] = NIL; L.prev[0] = NIL;
    L.dead[0] = 1; /* sentinel never counts as visible */
    L.cur = 0; L.cnt = 0;
    uint64_t vis = 0;
    uint32_t n = 0;
    int64_t rc = 0;

#define INSERT_RUN(POS, SRC, LEN)                                                  \
    do {                                                                           \
        if (rl_seek(&L, (POS))) { rc = -1; goto done; }                            \
        uint32_t left = L.cur, right = L.next[left];                               \
        for (size_t k = 0; k < (LEN); ++k) {                                       \
            uint32_t id = ++n;                                                     \
            parent[id - 1] = left; oright[id - 1] = right; lamport[id - 1] = id;   \
            agent[id - 1] = 0; deleted[id - 1] = 0; cp[id - 1] = (SRC)[k];         \
            L.next[id] = L.next[left]; L.prev[id] = left;                          \
            if (L.next[left] != NIL) L.prev[L.next[left]] = id;                    \
            L.next[left] = id; L.dead[id] = 0;                                     \
            left = id;                                                             \
        }                                                                          \
        L.cur = left; L.cnt = (POS) + (LEN); vis += (LEN);                         \
    } while (0)

    if (p->start_n) INSERT_RUN(0, p->start_cp, p->start_n);
    for (size_t i = 0; i < p->npatch; ++i) {
        uint64_t pos = p->pos[i], del = p->del[i];
        if (pos > vis || del > vis - pos) { rc = -1; goto done; }
        if (del) { /* remove(pos..pos+del): tombstone the visible items there */
            if (rl_seek(&L, pos + 1)) { rc = -1; goto done; }
            uint32_t c = L.cur;
            for (uint64_t k = 0; k < del; ++k) {
                while (L.dead[c]) c = L.next[c];
                L.dead[c] = 1; deleted[c - 1] = 1;
                if (k + 1 < del) c = L.next[c];
            }
            L.cur = c; L.cnt = pos; vis -= del;
        }
        if (p->ins_len[i]) INSERT_RUN(pos, p->ins_cp + p->ins_off[i], p->ins_len[i]);
    }
    rc = n;
#undef INSERT_RUN
done:
    free(L.next); free(L.prev); free(L.dead);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* RGA merge: CSR children, sibling sort, iterative pre-order DFS, tombstone compaction.       */
/* ------------------------------------------------------------------------------------------ */
typedef struct { const uint32_t* lam; const uint16_t* ag; } keyctx;
static inline int ts_greater(const keyctx* k, uint32_t a, uint32_t b) { /* ts(a) > ts(b) */
    uint32_t la = k->lam[a - 1], lb = k->lam[b - 1];
    if (la != lb) return la > lb;
    return k->ag[a - 1] > k->ag[b - 1];
}

int64_t orc_merge_rga(uint32_t n, const uint32_t* parent, const uint32_t* lamport,
                      const uint16_t* agent, const uint8_t* deleted, const uint32_t* cp,
                      uint8_t* out, size_t cap, uint32_t* order) {
    keyctx K = {lamport, agent};
    uint32_t* start = (uint32_t*)calloc((size_t)n + 2, 4);
    uint32_t* kids = (uint32_t*)malloc(((size_t)n + 1) * 4);
    uint32_t* stack = (uint32_t*)malloc(((size_t)n + 1) * 4);
    int64_t rc = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        uint32_t pr = parent[i - 1];
        if (pr > n || pr == i) { rc = -1; goto done; }
        start[pr + 1]++;
    }
    for (uint32_t v = 0; v <= n; ++v) start[v + 1] += start[v];
    {
        uint32_t* fill = (uint32_t*)malloc(((size_t)n + 1) * 4);
        memcpy(fill, start, ((size_t)n + 1) * 4);
        for (uint32_t i = 1; i <= n; ++i) kids[fill[parent[i - 1]]++] = i;
        free(fill);
    }
    /* sort each sibling group by timestamp ascending (stack pops the greatest first) */
    for (uint32_t v = 0; v <= n; ++v) {
        uint32_t a = start[v], b = start[v + 1];
        for (uint32_t i = a + 1; i < b; ++i) {
            uint32_t x = kids[i];
            uint32_t j = i;
            while (j > a && ts_greater(&K, kids[j - 1], x)) { kids[j] = kids[j - 1]; --j; }
            kids[j] = x;
        }
    }
    {
        size_t sp = 0, k = 0, visited = 0;
        stack[sp++] = 0;
        while (sp) {
            uint32_t v = stack[--sp];
            if (v) {
                if (order) order[visited] = v;
                visited++;
                if (!deleted[v - 1]) {
                    if (k + len1(cp[v - 1]) > cap) { rc = -2; goto done; }
                    k += enc1(cp[v - 1], out + k);
                }
            }
            for (uint32_t i = start[v]; i < start[v + 1]; ++i) stack[sp++] = kids[i];
        }
        if (visited != n) { rc = -1; goto done; } /* unreachable items: a cycle */
        rc = (int64_t)k;
    }
done:
    free(start); free(kids); free(stack);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Fugue: resolver with left/right anchors, and the in-order merge.                            */
/* ------------------------------------------------------------------------------------------ */
int64_t orc_resolve_fugue(const orc_patches* p, uint32_t* parent, uint8_t* side,
                          uint32_t* lamport, uint16_t* agent, uint8_t* deleted, uint32_t* cp) {
    size_t total = p->start_n;
    for (size_t i = 0; i < p->npatch; ++i) total += p->ins_len[i];
    rlist L;
    L.next = (uint32_t*)malloc((total + 1) * 4);
    L.prev = (uint32_t*)malloc((total + 1) * 4);
    L.dead = (uint8_t*)calloc(total + 1, 1);
    uint8_t* hasright = (uint8_t*)calloc(total + 1, 1);
    L.next[0] = NIL; L.prev[0] = NIL;
    L.dead[0] = 1;
    L.cur = 0; L.cnt = 0;
    uint64_t vis = 0;
    uint32_t n = 0;
    int64_t rc = 0;
    /* one item after `left`: right child of left if left has none yet, else left child of the
     * item that follows left in the full list */
#define FUGUE_RUN(POS, SRC, LEN)                                                   \
    do {                                                                           \
        if (rl_seek(&L, (POS))) { rc = -1; goto done; }                            \
        uint32_t left = L.cur;                                                     \
        for (size_t k = 0; k < (LEN); ++k) {                                       \
            uint32_t id = ++n, right = L.next[left];                               \
            if (!hasright[left]) {                                                 \
                parent[id - 1] = left; side[id - 1] = 0; hasright[left] = 1;       \
            } else {                                                               \
                if (right == NIL) { rc = -1; goto done; }                          \
                parent[id - 1] = right; side[id - 1] = 1;                          \
            }                                                                      \
            lamport[id - 1] = id; agent[id - 1] = 0; deleted[id - 1] = 0;          \
            cp[id - 1] = (SRC)[k];                                                 \
            L.next[id] = right; L.prev[id] = left;                                 \
            if (right != NIL) L.prev[right] = id;                                  \
            L.next[left] = id; L.dead[id] = 0;                                     \
            left = id;                                                             \
        }                                                                          \
        L.cur = left; L.cnt = (POS) + (LEN); vis += (LEN);                         \
    } while (0)
    if (p->start_n) FUGUE_RUN(0, p->start_cp, p->start_n);
    for (size_t i = 0; i < p->npatch; ++i) {
        uint64_t pos = p->pos[i], del = p->del[i];
        if (pos > vis || del > vis - pos) { rc = -1; goto done; }
        if (del) {
            if (rl_seek(&L, pos + 1)) { rc = -1; goto done; }
            uint32_t c = L.cur;
            for (uint64_t k = 0; k < del; ++k) {
                while (L.dead[c]) c = L.next[c];
                L.dead[c] = 1; deleted[c - 1] = 1;
                if (k + 1 < del) c = L.next[c];
            }
            L.cur = c; L.cnt = pos; vis -= del;
        }
        if (p->ins_len[i]) FUGUE_RUN(pos, p->ins_cp + p->ins_off[i], p->ins_len[i]);
    }
    rc = n;
#undef FUGUE_RUN
done:
    free(L.next); free(L.prev); free(L.dead); free(hasright);
    return rc;
}

int64_t orc_merge_fugue(uint32_t n, const uint32_t* parent, const uint8_t* side,
                        const uint32_t* lamport, const uint16_t* agent, const uint8_t* deleted,
                        const uint32_t* cp, uint8_t* out, size_t cap, uint32_t* order) {
    keyctx K = {lamport, agent};
    /* children of v: CSR over groups 2v (left children) and 2v + 1 (right children), each
     * ascending by timestamp */
    uint32_t* start = (uint32_t*)calloc(2 * (size_t)n + 3, 4);
    uint32_t* kids = (uint32_t*)malloc(((size_t)n + 1) * 4);
    /* the stack holds items to expand and (id | EMIT) markers: at most 2n + 1 entries */
    uint32_t* stack = (uint32_t*)malloc((2 * (size_t)n + 2) * 4);
    const uint32_t EMIT = 0x80000000u;
    int64_t rc = 0;
    if (n >= EMIT) { rc = -1; goto done; }
    for (uint32_t i = 1; i <= n; ++i) {
        uint32_t pr = parent[i - 1];
        if (pr > n || pr == i || (pr == 0 && side[i - 1])) { rc = -1; goto done; }
        start[2 * pr + (side[i - 1] ? 0 : 1) + 1]++;
    }
    for (uint32_t g = 0; g < 2 * n + 2; ++g) start[g + 1] += start[g];
    {
        uint32_t* fill = (uint32_t*)malloc((2 * (size_t)n + 2) * 4);
        memcpy(fill, start, (2 * (size_t)n + 2) * 4);
        for (uint32_t i = 1; i <= n; ++i) kids[fill[2 * parent[i - 1] + (side[i - 1] ? 0 : 1)]++] = i;
        free(fill);
    }
    for (uint32_t g = 0; g < 2 * n + 2; ++g) {
        uint32_t a = start[g], b = start[g + 1];
        for (uint32_t i = a + 1; i < b; ++i) {
            uint32_t x = kids[i];
            uint32_t j = i;
            while (j > a && ts_greater(&K, kids[j - 1], x)) { kids[j] = kids[j - 1]; --j; }
            kids[j] = x;
        }
    }
    {
        size_t sp = 0, k = 0, visited = 0;
        stack[sp++] = 0;
        while (sp) {
            uint32_t e = stack[--sp];
            if (e & EMIT) {
                uint32_t v = e & ~EMIT;
                if (order) order[visited] = v;
                visited++;
                if (!deleted[v - 1]) {
                    if (k + len1(cp[v - 1]) > cap) { rc = -2; goto done; }
                    k += enc1(cp[v - 1], out + k);
                }
                continue;
            }
            /* expand e: pushed in reverse of the walk (right children, e itself, left
             * children, each group ascending), so that the greatest left child pops first,
             * then e, then the greatest right child */
            for (uint32_t i = start[2 * e + 1]; i < start[2 * e + 2]; ++i) stack[sp++] = kids[i];
            if (e) stack[sp++] = e | EMIT;
            for (uint32_t i = start[2 * e]; i < start[2 * e + 1]; ++i) stack[sp++] = kids[i];
        }
        if (visited != n) { rc = -1; goto done; }
        rc = (int64_t)k;
    }
done:
    free(start); free(kids); free(stack);
    return rc;
}

/* Independent O(n^2) integrator (textbook RGA: skip successors with a greater timestamp). */
static int cmp_lam_idx(const void* a, const void* b, void* ctx) {
    const keyctx* k = (const keyctx*)ctx;
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    if (ts_greater(k, x, y)) return 1;
    if (ts_greater(k, y, x)) return -1;
    return 0;
}
static keyctx* g_sortctx;
static int cmp_tramp(const void* a, const void* b) { return cmp_lam_idx(a, b, g_sortctx); }

int64_t orc_merge_rga_naive(uint32_t n, const uint32_t* parent, const uint32_t* lamport,
                            const uint16_t* agent, const uint8_t* deleted, const uint32_t* cp,
                            uint8_t* out, size_t cap) {
    keyctx K = {lamport, agent};
    uint32_t* ord = (uint32_t*)malloc(((size_t)n + 1) * 4);
    uint32_t* next = (uint32_t*)malloc(((size_t)n + 1) * 4);
    uint8_t* placed = (uint8_t*)calloc((size_t)n + 1, 1);
    int64_t rc = 0;
    for (uint32_t i = 0; i < n; ++i) ord[i] = i + 1;
    g_sortctx = &K;
    qsort(ord, n, 4, cmp_tramp); /* causal order: lamport ascending */
    next[0] = NIL;
    placed[0] = 1;
    for (uint32_t t = 0; t < n; ++t) {
        uint32_t x = ord[t], p = parent[x - 1];
        if (p > n || !placed[p]) { rc = -1; goto done; }
        uint32_t at = p;
        while (next[at] != NIL && ts_greater(&K, next[at], x)) at = next[at];
        next[x] = next[at];
        next[at] = x;
        placed[x] = 1;
    }
    {
        size_t k = 0;
        for (uint32_t v = next[0]; v != NIL; v = next[v]) {
            if (deleted[v - 1]) continue;
            if (k + len1(cp[v - 1]) > cap) { rc = -2; goto done; }
            k += enc1(cp[v - 1], out + k);
        }
        rc = (int64_t)k;
    }
done:
    free(ord); free(next); free(placed);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Batched CPU baseline: one log per task, `threads` worker threads.                            */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_log* logs;
    uint32_t nlogs;
    uint64_t* digests;
    uint64_t* lens;
    volatile uint32_t* next_task;
    pthread_mutex_t* mu;
    int err;
} mm_job;

static void* mm_worker(void* arg) {
    mm_job* j = (mm_job*)arg;
    uint8_t* buf = NULL;
    size_t bcap = 0;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint32_t t = (*j->next_task)++;
        pthread_mutex_unlock(j->mu);
        if (t >= j->nlogs) break;
        const orc_log* L = &j->logs[t];
        size_t need = (size_t)L->n * 4 + 4;
        if (need > bcap) { free(buf); buf = (uint8_t*)malloc(need); bcap = need; }
        int64_t k = orc_merge_rga(L->n, L->parent, L->lamport, L->agent, L->deleted, L->cp, buf,
                                  bcap, NULL);
        if (k < 0) { j->err = (int)k; break; }
        j->lens[t] = (uint64_t)k;
        j->digests[t] = orc_tree_digest(buf, (size_t)k);
    }
    free(buf);
    return NULL;
}

int orc_merge_many(const orc_log* logs, uint32_t nlogs, int threads, uint64_t* digests,
                   uint64_t* lens) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    mm_job* jobs = (mm_job*)malloc(sizeof(mm_job) * (size_t)threads);
    volatile uint32_t next_task = 0;
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    for (int i = 0; i < threads; ++i) {
        jobs[i] = (mm_job){logs, nlogs, digests, lens, &next_task, &mu, 0};
        pthread_create(&th[i], NULL, mm_worker, &jobs[i]);
    }
    int err = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        if (jobs[i].err) err = jobs[i].err;
    }
    free(th); free(jobs);
    return err;
}

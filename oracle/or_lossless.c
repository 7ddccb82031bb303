/* oracle/or_lossless.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of zenwebp 0.2.0's VP8L encoder (src/encoder/api.rs), used for
 * the ALPH chunk of lossy-with-alpha images (encode_alpha_lossless, :1175-1222)
 * and for lossless WebPEncoder output (encode_frame_lossless, :945-1173):
 * subtract-green + (optional) "left/top" predictor transform, one Huffman group,
 * no color cache, no backward references except same-pixel runs.
 *
 * The Huffman construction follows build_huffman_tree (:163-287) including the
 * tie behaviour of Rust's std BinaryHeap (from_iter = rebuild, pop =
 * sift_down_to_bottom + sift_up, PeekMut write-back = sift_down), restated
 * below.  When a tree exceeds the length limit (15, or 7 for the code-length
 * code), the reference re-assigns lengths in the order of
 * `sort_unstable_by_key(frequency)` (:259-260), whose order among EQUAL
 * frequencies is that of the Rust standard library's unstable sort (ipnsort,
 * rust-version 1.92 in Cargo.toml); rust_sort_unstable_by_key below restates
 * it.  No Rust toolchain is available here, so that restatement is checked by
 * its invariants (tests/test_lossless.py), not against Rust's own output.
 */
#include <stdlib.h>
#include <string.h>

#include "zw_oracle.h"

/* BitWriter (:110-148) */
typedef struct {
    uint8_t *buf;
    size_t len, cap;
    uint64_t acc;
    unsigned nbits;
} bw_t;

static int bw_put8(bw_t *w, const uint8_t *p, size_t n)
{
    if (w->len + n > w->cap) {
        size_t c = w->cap ? w->cap * 2 : 1024;
        while (c < w->len + n) c *= 2;
        uint8_t *nb = (uint8_t *)realloc(w->buf, c);
        if (!nb) return -1;
        w->buf = nb;
        w->cap = c;
    }
    memcpy(w->buf + w->len, p, n);
    w->len += n;
    return 0;
}
static void bw_write(bw_t *w, uint64_t bits, unsigned nbits)
{
    w->acc |= bits << w->nbits; /* w->nbits < 64 */
    w->nbits += nbits;
    if (w->nbits >= 64) {
        uint8_t b[8];
        for (int i = 0; i < 8; i++) b[i] = (uint8_t)(w->acc >> (8 * i));
        bw_put8(w, b, 8);
        w->nbits -= 64;
        unsigned sh = nbits - w->nbits; /* bits.checked_shr(sh).unwrap_or(0) */
        w->acc = sh >= 64 ? 0 : bits >> sh;
    }
}
static void bw_flush(bw_t *w)
{
    if (w->nbits % 8) bw_write(w, 0, 8 - w->nbits % 8);
    if (w->nbits > 0) {
        uint8_t b[8];
        for (int i = 0; i < 8; i++) b[i] = (uint8_t)(w->acc >> (8 * i));
        bw_put8(w, b, w->nbits / 8);
        w->acc = 0;
        w->nbits = 0;
    }
}

/* write_single_entry_huffman_tree (:152-161) */
static void single_tree(bw_t *w, unsigned sym)
{
    bw_write(w, 1, 2);
    if (sym <= 1) {
        bw_write(w, 0, 1);
        bw_write(w, sym, 1);
    } else {
        bw_write(w, 1, 1);
        bw_write(w, sym, 8);
    }
}

/* --- Rust std::collections::BinaryHeap<Item> with Item ordered by REVERSED
 * frequency (a max-heap on Ord = a min-heap on frequency).  "a <= b" in Ord is
 * a.f >= b.f. */
typedef struct {
    uint32_t f;
    uint16_t i;
} item_t;
static int ord_le(item_t a, item_t b) { return a.f >= b.f; } /* a <= b */
static int ord_lt(item_t a, item_t b) { return a.f > b.f; }  /* a < b  */
static int ord_ge(item_t a, item_t b) { return a.f <= b.f; } /* a >= b */

/* sift_down_range(pos, end) */
static void heap_sift_down_range(item_t *d, size_t pos, size_t end)
{
    item_t el = d[pos];
    size_t hole = pos, child = 2 * hole + 1;
    while (child + 2 <= end) { /* child <= end.saturating_sub(2) */
        child += ord_le(d[child], d[child + 1]) ? 1 : 0;
        if (ord_ge(el, d[child])) {
            d[hole] = el;
            return;
        }
        d[hole] = d[child];
        hole = child;
        child = 2 * hole + 1;
    }
    if (end >= 1 && child == end - 1 && ord_lt(el, d[child])) {
        d[hole] = d[child];
        hole = child;
    }
    d[hole] = el;
}
/* sift_up(start, pos) */
static void heap_sift_up(item_t *d, size_t start, size_t pos)
{
    item_t el = d[pos];
    size_t hole = pos;
    while (hole > start) {
        size_t parent = (hole - 1) / 2;
        if (ord_le(el, d[parent])) break;
        d[hole] = d[parent];
        hole = parent;
    }
    d[hole] = el;
}
/* sift_down_to_bottom(0) on a heap of length n */
static void heap_sift_down_to_bottom(item_t *d, size_t n)
{
    item_t el = d[0];
    size_t hole = 0, child = 1;
    while (child + 2 <= n) {
        child += ord_le(d[child], d[child + 1]) ? 1 : 0;
        d[hole] = d[child];
        hole = child;
        child = 2 * hole + 1;
    }
    if (n >= 1 && child == n - 1) {
        d[hole] = d[child];
        hole = child;
    }
    d[hole] = el;
    heap_sift_up(d, 0, hole);
}
/* pop(): swap the last into the root, sift_down_to_bottom */
static item_t heap_pop(item_t *d, size_t *n)
{
    item_t last = d[--*n];
    if (*n == 0) return last;
    item_t top = d[0];
    d[0] = last;
    heap_sift_down_to_bottom(d, *n);
    return top;
}

/* --- Rust 1.92 `<[T]>::sort_unstable_by_key` for T = (usize, u32) keyed by
 * the u32 (core::slice::sort::unstable).  Only the order among equal keys
 * matters here, so every step that can move equal keys is restated as is:
 *   sort():      len <= 20 -> insertion sort (stable); else ipnsort()
 *   ipnsort():   a leading run covering the whole slice is kept (reversed if
 *                strictly descending); else quicksort(limit = 2*ilog2(len|1))
 *   quicksort(): len <= 32 -> small_sort_general (sort4/sort8_stable +
 *                insert_tail + bidirectional_merge: a stable sort for a total
 *                order, so insertion sort gives the same result for 16-byte
 *                T, which has no "efficient in-place swap");
 *                limit exhausted -> heapsort; pivot = median3 / recursive
 *                pseudo-median of 3 (shared/pivot.rs); if the ancestor pivot
 *                is not less than the pivot, partition by <= and drop the
 *                equal part; partition = swap pivot to 0, branchless cyclic
 *                Lomuto over v[1..], swap pivot into place.  */
typedef struct {
    uint32_t idx, key;
} kv_t;

static void kv_insertion(kv_t *v, size_t n)
{
    for (size_t i = 1; i < n; i++) {
        kv_t t = v[i];
        size_t j = i;
        while (j > 0 && t.key < v[j - 1].key) {
            v[j] = v[j - 1];
            j--;
        }
        v[j] = t;
    }
}

static void kv_sift_down(kv_t *v, size_t n, size_t node)
{
    for (;;) {
        size_t child = 2 * node + 1;
        if (child >= n) break;
        if (child + 1 < n) child += v[child].key < v[child + 1].key;
        if (!(v[node].key < v[child].key)) break;
        kv_t t = v[node];
        v[node] = v[child];
        v[child] = t;
        node = child;
    }
}

static void kv_heapsort(kv_t *v, size_t n)
{
    for (size_t i = n + n / 2; i-- > 0;) {
        size_t sift = 0;
        if (i >= n) {
            sift = i - n;
        } else {
            kv_t t = v[0];
            v[0] = v[i];
            v[i] = t;
        }
        kv_sift_down(v, i < n ? i : n, sift);
    }
}

static size_t kv_median3(const kv_t *v, size_t a, size_t b, size_t c)
{
    int x = v[a].key < v[b].key, y = v[a].key < v[c].key;
    if (x == y) return ((v[b].key < v[c].key) ^ x) ? c : b;
    return a;
}

static size_t kv_median3_rec(const kv_t *v, size_t a, size_t b, size_t c, size_t n)
{
    if (n * 8 >= 64) {
        size_t n8 = n / 8;
        a = kv_median3_rec(v, a, a + n8 * 4, a + n8 * 7, n8);
        b = kv_median3_rec(v, b, b + n8 * 4, b + n8 * 7, n8);
        c = kv_median3_rec(v, c, c + n8 * 4, c + n8 * 7, n8);
    }
    return kv_median3(v, a, b, c);
}

static size_t kv_choose_pivot(const kv_t *v, size_t n)
{
    size_t n8 = n / 8;
    if (n < 64) return kv_median3(v, 0, n8 * 4, n8 * 7);
    return kv_median3_rec(v, 0, n8 * 4, n8 * 7, n8);
}

/* partition(): `le` selects the `!is_less(pivot, x)` predicate (x <= pivot) */
static size_t kv_partition(kv_t *v, size_t n, size_t p, int le)
{
    kv_t t = v[0];
    v[0] = v[p];
    v[p] = t;
    const uint32_t pk = v[0].key;
    kv_t *w = v + 1;
    const size_t m = n - 1;
    size_t num_lt = 0;
    if (m > 0) {
        /* cyclic Lomuto: the hole starts at w[0] (its value saved) and
         * every element w[1..m), then the saved one, is placed in turn */
        const kv_t saved = w[0];
        size_t gap = 0;
        for (size_t r = 1; r <= m; r++) {
            const kv_t e = r < m ? w[r] : saved;
            const int is_lt = le ? !(pk < e.key) : e.key < pk;
            w[gap] = w[num_lt];
            w[num_lt] = e;
            gap = r < m ? r : gap;
            num_lt += (size_t)is_lt;
        }
    }
    t = v[0];
    v[0] = v[num_lt];
    v[num_lt] = t;
    return num_lt;
}

static void kv_quicksort(kv_t *v, size_t n, const kv_t *ancestor, uint32_t limit)
{
    for (;;) {
        if (n <= 32) {
            kv_insertion(v, n);
            return;
        }
        if (limit == 0) {
            kv_heapsort(v, n);
            return;
        }
        limit--;
        size_t p = kv_choose_pivot(v, n);
        if (ancestor && !(ancestor->key < v[p].key)) {
            size_t num_le = kv_partition(v, n, p, 1);
            v += num_le + 1;
            n -= num_le + 1;
            ancestor = NULL;
            continue;
        }
        size_t num_lt = kv_partition(v, n, p, 0);
        kv_quicksort(v, num_lt, ancestor, limit);
        ancestor = &v[num_lt];
        v += num_lt + 1;
        n -= num_lt + 1;
    }
}

void or_rust_sort_unstable_by_key(uint32_t *idx, uint32_t *key, size_t n)
{
    if (n < 2) return;
    kv_t *v = (kv_t *)malloc(sizeof(kv_t) * n);
    for (size_t i = 0; i < n; i++) v[i] = (kv_t){idx[i], key[i]};
    if (n <= 20) {
        kv_insertion(v, n);
    } else {
        size_t run = 2;
        const int desc = v[1].key < v[0].key;
        if (desc)
            while (run < n && v[run].key < v[run - 1].key) run++;
        else
            while (run < n && !(v[run].key < v[run - 1].key)) run++;
        if (run == n) {
            if (desc)
                for (size_t i = 0; i < n / 2; i++) {
                    kv_t t = v[i];
                    v[i] = v[n - 1 - i];
                    v[n - 1 - i] = t;
                }
        } else {
            uint32_t lg = 0;
            for (size_t x = n | 1; x > 1; x >>= 1) lg++;
            kv_quicksort(v, n, NULL, 2 * lg);
        }
    }
    for (size_t i = 0; i < n; i++) {
        idx[i] = v[i].idx;
        key[i] = v[i].key;
    }
    free(v);
}

/* build_huffman_tree (:163-287) */
static int build_tree(const uint32_t *freq, int n, uint8_t *len, uint16_t *code, int limit)
{
    int nz = 0;
    for (int i = 0; i < n; i++) nz += freq[i] > 0;
    if (nz <= 1) {
        memset(len, 0, (size_t)n);
        memset(code, 0, (size_t)n * 2);
        return 0;
    }
    item_t *h = (item_t *)malloc(sizeof(item_t) * (size_t)nz);
    uint16_t(*internal)[2] = (uint16_t(*)[2])malloc(sizeof(uint16_t) * 2 * (size_t)nz);
    size_t hn = 0, ni = 0;
    for (int i = 0; i < n; i++)
        if (freq[i] > 0) h[hn++] = (item_t){freq[i], (uint16_t)i};
    for (size_t k = hn / 2; k > 0; k--) heap_sift_down_range(h, k - 1, hn); /* rebuild */
    while (hn > 1) {
        item_t a = heap_pop(h, &hn);
        /* peek_mut: root = Item(a.f + root.f, new internal node); sift_down(0) */
        internal[ni][0] = a.i;
        internal[ni][1] = h[0].i;
        ni++;
        h[0] = (item_t){a.f + h[0].f, (uint16_t)(ni + (size_t)n - 1)};
        heap_sift_down_range(h, 0, hn);
    }
    /* depths */
    memset(len, 0, (size_t)n);
    {
        int cap = 2 * n + 8, sp = 0;
        int(*st)[2] = (int(*)[2])malloc(sizeof(int) * 2 * (size_t)cap);
        st[sp][0] = h[0].i;
        st[sp][1] = 0;
        sp++;
        while (sp > 0) {
            sp--;
            int node = st[sp][0], depth = st[sp][1];
            if (node < n) {
                len[node] = (uint8_t)depth;
            } else {
                st[sp][0] = internal[node - n][0];
                st[sp][1] = depth + 1;
                sp++;
                st[sp][0] = internal[node - n][1];
                st[sp][1] = depth + 1;
                sp++;
            }
        }
        free(st);
    }
    free(h);
    free(internal);
    /* limit the code lengths */
    int maxl = 0;
    for (int i = 0; i < n; i++) maxl = len[i] > maxl ? len[i] : maxl;
    if (maxl > limit) {
        uint32_t counts[16] = {0};
        for (int i = 0; i < n; i++) counts[len[i] < limit ? len[i] : limit]++;
        uint32_t total = 0;
        for (int i = 1; i <= limit; i++) total += counts[i] << (limit - i);
        while (total > (1u << limit)) {
            int i = limit - 1;
            while (counts[i] == 0) i--;
            counts[i]--;
            counts[limit]--;
            counts[i + 1] += 2;
            total--;
        }
        /* indexes = frequencies.enumerate(); sort_unstable_by_key(frequency) */
        uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n);
        uint32_t *key = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n);
        for (int i = 0; i < n; i++) {
            idx[i] = (uint32_t)i;
            key[i] = freq[i];
        }
        or_rust_sort_unstable_by_key(idx, key, (size_t)n);
        int l = limit;
        for (int k = 0; k < n; k++) {
            if (key[k] > 0) {
                while (counts[l] == 0) l--;
                len[idx[k]] = (uint8_t)l;
                counts[l]--;
            }
        }
        free(idx);
        free(key);
    }
    /* canonical codes, bit-reversed */
    memset(code, 0, (size_t)n * 2);
    uint32_t c = 0;
    for (int l = 1; l <= limit; l++) {
        for (int i = 0; i < n; i++)
            if (len[i] == l) {
                uint16_t v = (uint16_t)c, r = 0;
                for (int b = 0; b < 16; b++) r |= (uint16_t)(((v >> b) & 1) << (15 - b));
                code[i] = (uint16_t)(r >> (16 - l));
                c++;
            }
        c <<= 1;
    }
    return 1;
}

/* write_huffman_tree (:289-364) */
static void write_tree(bw_t *w, const uint32_t *freq, int n, uint8_t *len, uint16_t *code)
{
    if (!build_tree(freq, n, len, code, 15)) {
        int sym = 0;
        for (int i = 0; i < n; i++)
            if (freq[i] > 0) {
                sym = i;
                break;
            }
        single_tree(w, (unsigned)(uint8_t)sym);
        return;
    }
    uint8_t cll[16];
    uint16_t clc[16];
    uint32_t clf[16] = {0};
    for (int i = 0; i < n; i++) clf[len[i]]++;
    const int single = !build_tree(clf, 16, cll, clc, 7);
    static const int ORDER[19] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    bw_write(w, 0, 1);
    bw_write(w, 19 - 4, 4);
    for (int k = 0; k < 19; k++) {
        int i = ORDER[k];
        if (i > 15 || clf[i] == 0) bw_write(w, 0, 3);
        else if (single) bw_write(w, 1, 3);
        else bw_write(w, cll[i], 3);
    }
    if (n == 256) {
        bw_write(w, 1, 1);
        bw_write(w, 3, 3);
        bw_write(w, 254, 8);
    } else {
        bw_write(w, 0, 1); /* 280 */
    }
    if (!single)
        for (int i = 0; i < n; i++) bw_write(w, clc[len[i]], cll[len[i]]);
}

/* length_to_symbol (:355-362) */
static void len_sym(unsigned run, unsigned *sym, unsigned *extra)
{
    unsigned l = run - 1, hb = 31 - (unsigned)__builtin_clz(l);
    unsigned second = (l >> (hb - 1)) & 1;
    *extra = hb - 1;
    *sym = 2 * hb + second;
}

/* run length after pixel p (count_run / write_run, :366-417): up to 4096
 * following pixels equal to p */
static size_t run_after(const uint8_t *px, size_t np, size_t p)
{
    size_t r = 0;
    while (r < 4096 && p + 1 + r < np && memcmp(px + 4 * (p + 1 + r), px + 4 * p, 4) == 0) r++;
    return r;
}

int or_encode_frame_lossless(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color,
                             int use_predictor, int implicit_dims, uint8_t **out, size_t *out_len)
{
    static const int BPP[4] = {1, 2, 3, 4};
    *out = NULL;
    *out_len = 0;
    if (color < 0 || color > 3) return OR_EINVAL;
    const int bpp = BPP[color];
    const int is_color = color >= 2, is_alpha = color == 1 || color == 3;
    if ((uint64_t)width * height * (uint64_t)bpp != (uint64_t)len) return OR_EINVALID_BUFFER_SIZE; /* assert_eq (panic) */
    if (width == 0 || width > 16384 || height == 0 || height > 16384) return OR_EINVALID_DIMENSIONS;
    bw_t w = {0};
    if (!implicit_dims) {
        bw_write(&w, 0x2f, 8);
        bw_write(&w, width - 1, 14);
        bw_write(&w, height - 1, 14);
        bw_write(&w, (uint64_t)is_alpha, 1);
        bw_write(&w, 0, 3);
    }
    bw_write(&w, 5, 3); /* subtract green */
    if (use_predictor) {
        bw_write(&w, 0x39, 6);
        bw_write(&w, 0, 1);
        single_tree(&w, 2);
        for (int i = 0; i < 4; i++) single_tree(&w, 0);
    }
    bw_write(&w, 0, 1);
    bw_write(&w, 0, 1);
    bw_write(&w, 0, 1);
    const size_t np = (size_t)width * height;
    uint8_t *px = (uint8_t *)malloc(np * 4);
    if (!px) return OR_EINVAL;
    for (size_t i = 0; i < np; i++) {
        const uint8_t *s = data + i * bpp;
        uint8_t *d = px + 4 * i;
        switch (color) {
        case 0: d[0] = d[1] = d[2] = s[0]; d[3] = 255; break;
        case 1: d[0] = d[1] = d[2] = s[0]; d[3] = s[1]; break;
        case 2: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255; break;
        default: memcpy(d, s, 4); break;
        }
        d[0] = (uint8_t)(d[0] - d[1]);
        d[2] = (uint8_t)(d[2] - d[1]);
    }
    if (use_predictor) {
        const size_t rb = (size_t)width * 4;
        for (size_t y = height - 1; y >= 1; y--)
            for (size_t i = 0; i < rb; i++) px[y * rb + i] = (uint8_t)(px[y * rb + i] - px[(y - 1) * rb + i]);
        for (size_t i = rb - 1; i >= 4; i--) px[i] = (uint8_t)(px[i] - px[i - 4]);
        px[3] = (uint8_t)(px[3] - 255);
    }
    uint32_t f0[256] = {0}, f1[280] = {0}, f2[256] = {0}, f3[256] = {0};
    if (color == 0) f0[0] = f2[0] = f3[0] = 1;
    if (color == 1) f0[0] = f2[0] = 1;
    if (color == 2) f3[0] = 1;
    for (size_t p = 0; p < np;) {
        const uint8_t *q = px + 4 * p;
        f1[q[1]]++;
        if (is_color) {
            f0[q[0]]++;
            f2[q[2]]++;
        }
        if (is_alpha) f3[q[3]]++;
        size_t r = run_after(px, np, p);
        if (r > 0) {
            if (r <= 4) f1[256 + r - 1]++;
            else {
                unsigned s, e;
                len_sym((unsigned)r, &s, &e);
                f1[256 + s]++;
            }
        }
        p += 1 + r;
    }
    uint8_t l0[256] = {0}, l1[280] = {0}, l2[256] = {0}, l3[256] = {0};
    uint16_t c0[256] = {0}, c1[280] = {0}, c2[256] = {0}, c3[256] = {0};
    write_tree(&w, f1, 280, l1, c1);
    if (is_color) {
        write_tree(&w, f0, 256, l0, c0);
        write_tree(&w, f2, 256, l2, c2);
    } else {
        single_tree(&w, 0);
        single_tree(&w, 0);
    }
    if (is_alpha) write_tree(&w, f3, 256, l3, c3);
    else if (use_predictor) single_tree(&w, 0);
    else single_tree(&w, 255);
    single_tree(&w, 1);
    for (size_t p = 0; p < np;) {
        const uint8_t *q = px + 4 * p;
        uint64_t code = c1[q[1]];
        unsigned n = l1[q[1]];
        if (is_color) {
            code |= (uint64_t)c0[q[0]] << n;
            n += l0[q[0]];
            code |= (uint64_t)c2[q[2]] << n;
            n += l2[q[2]];
        }
        if (is_alpha) {
            code |= (uint64_t)c3[q[3]] << n;
            n += l3[q[3]];
        }
        bw_write(&w, code, n);
        size_t r = run_after(px, np, p);
        if (r > 0) {
            if (r <= 4) bw_write(&w, c1[256 + r - 1], l1[256 + r - 1]);
            else {
                unsigned s, e;
                len_sym((unsigned)r, &s, &e);
                bw_write(&w, c1[256 + s], l1[256 + s]);
                bw_write(&w, (uint64_t)(r - 1) & ((1ull << e) - 1), e);
            }
        }
        p += 1 + r;
    }
    bw_flush(&w);
    free(px);
    *out = w.buf;
    *out_len = w.len;
    return OR_OK;
}

/* encode_alpha_lossless (:1175-1222): header byte (no preprocessing, no
 * filtering, compression 1) + the alpha plane as an L8 VP8L image with
 * implicit dimensions and default params (predictor on). */
int or_encode_alpha(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, uint8_t **out,
                    size_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    const int bpp = color == 1 ? 2 : (color == 3 ? 4 : 0);
    if (!bpp) return OR_EINVAL;
    if (width == 0 || width > 16384 || height == 0 || height > 16384) return OR_EINVALID_DIMENSIONS;
    const size_t np = (size_t)width * height;
    if (len != np * (size_t)bpp) return OR_EINVALID_BUFFER_SIZE;
    uint8_t *a = (uint8_t *)malloc(np ? np : 1);
    for (size_t i = 0; i < np; i++) a[i] = data[i * bpp + bpp - 1];
    uint8_t *body = NULL;
    size_t blen = 0;
    int rc = or_encode_frame_lossless(a, np, width, height, 0, 1, 1, &body, &blen);
    free(a);
    if (rc) return rc;
    uint8_t *o = (uint8_t *)malloc(blen + 1);
    o[0] = 1; /* preprocessing 0 << 4 | filtering 0 << 2 | compression 1 */
    memcpy(o + 1, body, blen);
    free(body);
    *out = o;
    *out_len = blen + 1;
    return OR_OK;
}


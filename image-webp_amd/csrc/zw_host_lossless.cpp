// zw_host_lossless.cpp -- host VP8L coder and the extended (VP8X) container.
//
// The lossless side of WebPEncoder::encode (encoder/api.rs:1291-1398):
//   * encode_frame_lossless (:945-1173): subtract-green + left/top predictor
//     transform, a single Huffman group (green+length 280 symbols, red, blue,
//     alpha, distance), no colour cache, no backward references other than
//     runs of the previous pixel (count_run / write_run, :366-417);
//   * encode_alpha_lossless (:1175-1222): the ALPH chunk every lossy RGBA / LA
//     encode carries -- the alpha plane as an L8 VP8L image with implicit
//     dimensions behind a one-byte header;
//   * the VP8X container with ICCP / ALPH / EXIF / XMP chunks (:1319-1395).
// Like the VP8 bool coder this is sequential entropy coding and stays on the
// host.  The Huffman builder reproduces build_huffman_tree (:163-287) including
// Rust's BinaryHeap tie behaviour (heapify, pop = sift to the bottom then up,
// peek_mut write-back = sift down), so equal frequencies resolve as in the
// reference.  Over-long trees (> 15 bits, > 7 for the code-length code) are
// re-balanced as the reference does, in the order of the reference's
// sort_unstable_by_key (Rust 1.92's ipnsort, restated in RustUnstableSort).
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "../../include/zwebp.h"
#include "zw_host_internal.h"

namespace {

class BitSink {
  public:
    explicit BitSink(std::vector<uint8_t>& o) : out_(o) {}
    // BitWriter::write_bits (:125-137): LSB-first into a 64-bit accumulator
    void put(uint64_t bits, unsigned n)
    {
        acc_ |= bits << fill_;
        fill_ += n;
        if (fill_ >= 64) {
            emit8();
            fill_ -= 64;
            const unsigned used = n - fill_;
            acc_ = used >= 64 ? 0 : bits >> used;
        }
    }
    void finish()  // BitWriter::flush (:139-148)
    {
        if (fill_ & 7) put(0, 8 - (fill_ & 7));
        for (unsigned i = 0; i < fill_ / 8; i++) out_.push_back((uint8_t)(acc_ >> (8 * i)));
        acc_ = 0;
        fill_ = 0;
    }

  private:
    void emit8()
    {
        for (int i = 0; i < 8; i++) out_.push_back((uint8_t)(acc_ >> (8 * i)));
    }
    std::vector<uint8_t>& out_;
    uint64_t acc_ = 0;
    unsigned fill_ = 0;
};

void put_single_symbol_code(BitSink& w, unsigned sym)  // write_single_entry_huffman_tree (:152-161)
{
    w.put(1, 2);
    if (sym <= 1) {
        w.put(0, 1);
        w.put(sym, 1);
    } else {
        w.put(1, 1);
        w.put(sym, 8);
    }
}

// Rust BinaryHeap<Item> where Item's Ord is the REVERSED frequency: the root is
// the smallest frequency.  `below(a, b)` is Ord's a < b, i.e. a.freq > b.freq.
struct Node {
    uint32_t freq;
    uint16_t id;
};
struct RustMinHeap {
    std::vector<Node> d;
    static bool below(const Node& a, const Node& b) { return a.freq > b.freq; }
    static bool not_above(const Node& a, const Node& b) { return a.freq >= b.freq; }  // a <= b
    void sift_down(size_t pos, size_t end)
    {
        const Node el = d[pos];
        size_t hole = pos, c = 2 * pos + 1;
        while (c + 2 <= end) {
            if (not_above(d[c], d[c + 1])) c++;
            if (!below(el, d[c])) {  // el >= child: in order
                d[hole] = el;
                return;
            }
            d[hole] = d[c];
            hole = c;
            c = 2 * hole + 1;
        }
        if (end && c == end - 1 && below(el, d[c])) {
            d[hole] = d[c];
            hole = c;
        }
        d[hole] = el;
    }
    void heapify()
    {
        for (size_t k = d.size() / 2; k-- > 0;) sift_down(k, d.size());
    }
    Node pop()
    {
        Node last = d.back();
        d.pop_back();
        if (d.empty()) return last;
        std::swap(last, d[0]);
        // sift_down_to_bottom(0) + sift_up(0, hole)
        const size_t n = d.size();
        const Node el = d[0];
        size_t hole = 0, c = 1;
        while (c + 2 <= n) {
            if (not_above(d[c], d[c + 1])) c++;
            d[hole] = d[c];
            hole = c;
            c = 2 * hole + 1;
        }
        if (c == n - 1) {
            d[hole] = d[c];
            hole = c;
        }
        while (hole > 0) {
            const size_t parent = (hole - 1) / 2;
            if (not_above(el, d[parent])) break;
            d[hole] = d[parent];
            hole = parent;
        }
        d[hole] = el;
        return last;
    }
};

// `indexes.sort_unstable_by_key(|&(_, f)| f)` (:259-260) on (symbol, freq)
// pairs.  The order among equal frequencies decides which tied symbols get the
// longer codes, so the Rust 1.92 standard library's unstable sort
// (core::slice::sort::unstable) is followed step by step: insertion sort up to
// 20 elements; a whole-slice leading run is kept (reversed when strictly
// descending); otherwise introsort-style quicksort with limit 2*ilog2(len|1),
// stable small sort at <= 32 elements (the 16-byte pair takes
// small_sort_general, a stable sort), heapsort once the limit is spent,
// (recursive) median-of-3 pivots, the equal-to-ancestor-pivot shortcut, and
// the branchless cyclic Lomuto partition.
class RustUnstableSort {
  public:
    struct Pair {
        uint16_t sym;
        uint32_t f;
    };
    static void sort(Pair* v, size_t n)
    {
        if (n < 2) return;
        if (n <= 20) return insertion(v, n);
        size_t run = 2;
        const bool desc = v[1].f < v[0].f;
        while (run < n && (desc ? v[run].f < v[run - 1].f : !(v[run].f < v[run - 1].f))) run++;
        if (run == n) {
            if (desc) std::reverse(v, v + n);
            return;
        }
        unsigned lg = 0;
        for (size_t x = n | 1; x > 1; x >>= 1) lg++;
        quick(v, n, nullptr, 2 * lg);
    }

  private:
    static void insertion(Pair* v, size_t n)
    {
        for (size_t i = 1; i < n; i++)
            for (size_t j = i; j > 0 && v[j].f < v[j - 1].f; j--) std::swap(v[j], v[j - 1]);
    }
    static void heapsort(Pair* v, size_t n)
    {
        for (size_t i = n + n / 2; i-- > 0;) {
            size_t node = i >= n ? i - n : 0;
            if (i < n) std::swap(v[0], v[i]);
            const size_t end = std::min(i, n);
            for (size_t c; (c = 2 * node + 1) < end; node = c) {
                if (c + 1 < end && v[c].f < v[c + 1].f) c++;
                if (!(v[node].f < v[c].f)) break;
                std::swap(v[node], v[c]);
            }
        }
    }
    static size_t med3(const Pair* v, size_t a, size_t b, size_t c)
    {
        const bool ab = v[a].f < v[b].f, ac = v[a].f < v[c].f;
        if (ab != ac) return a;
        return ((v[b].f < v[c].f) != ab) ? c : b;
    }
    static size_t med3_rec(const Pair* v, size_t a, size_t b, size_t c, size_t n)
    {
        if (n >= 8) {  // n * 8 >= 64
            const size_t s = n / 8;
            a = med3_rec(v, a, a + 4 * s, a + 7 * s, s);
            b = med3_rec(v, b, b + 4 * s, b + 7 * s, s);
            c = med3_rec(v, c, c + 4 * s, c + 7 * s, s);
        }
        return med3(v, a, b, c);
    }
    static size_t pivot(const Pair* v, size_t n)
    {
        const size_t s = n / 8;
        return n < 64 ? med3(v, 0, 4 * s, 7 * s) : med3_rec(v, 0, 4 * s, 7 * s, s);
    }
    // Pivot to the front, cyclic Lomuto over the rest (elements 1..n-1 then
    // the one first lifted out of the hole), pivot into place.
    static size_t partition(Pair* v, size_t n, size_t p, bool or_equal)
    {
        std::swap(v[0], v[p]);
        const uint32_t pf = v[0].f;
        Pair* w = v + 1;
        const size_t m = n - 1;
        size_t lt = 0;
        if (m) {
            const Pair lifted = w[0];
            size_t hole = 0;
            for (size_t r = 1; r <= m; r++) {
                const Pair e = r < m ? w[r] : lifted;
                w[hole] = w[lt];
                w[lt] = e;
                if (r < m) hole = r;
                lt += or_equal ? !(pf < e.f) : e.f < pf;
            }
        }
        std::swap(v[0], v[lt]);
        return lt;
    }
    static void quick(Pair* v, size_t n, const Pair* ancestor, unsigned limit)
    {
        for (;;) {
            if (n <= 32) return insertion(v, n);
            if (!limit) return heapsort(v, n);
            limit--;
            const size_t p = pivot(v, n);
            if (ancestor && !(ancestor->f < v[p].f)) {
                const size_t le = partition(v, n, p, true);
                v += le + 1;
                n -= le + 1;
                ancestor = nullptr;
                continue;
            }
            const size_t lt = partition(v, n, p, false);
            quick(v, lt, ancestor, limit);
            ancestor = v + lt;
            v += lt + 1;
            n -= lt + 1;
        }
    }
};

// build_huffman_tree (:163-287): returns false for <= 1 used symbol.
bool huffman_lengths_codes(const uint32_t* freq, int n, uint8_t* len, uint16_t* code, int limit)
{
    std::fill(len, len + n, 0);
    std::fill(code, code + n, 0);
    RustMinHeap h;
    for (int i = 0; i < n; i++)
        if (freq[i]) h.d.push_back({freq[i], (uint16_t)i});
    if (h.d.size() <= 1) return false;
    h.heapify();
    std::vector<std::pair<uint16_t, uint16_t>> inner;  // (popped, root) children of node n + k
    inner.reserve(h.d.size());
    while (h.d.size() > 1) {
        const Node a = h.pop();
        inner.emplace_back(a.id, h.d[0].id);
        h.d[0] = {a.freq + h.d[0].freq, (uint16_t)(inner.size() + (size_t)n - 1)};
        h.sift_down(0, h.d.size());
    }
    // depths (the walk order does not matter for lengths)
    std::vector<std::pair<int, int>> todo{{h.d[0].id, 0}};
    while (!todo.empty()) {
        auto [node, depth] = todo.back();
        todo.pop_back();
        if (node < n) {
            len[node] = (uint8_t)depth;
        } else {
            todo.emplace_back(inner[node - n].first, depth + 1);
            todo.emplace_back(inner[node - n].second, depth + 1);
        }
    }
    if (*std::max_element(len, len + n) > limit) {
        uint32_t cnt[16] = {0};
        for (int i = 0; i < n; i++) cnt[std::min<int>(len[i], limit)]++;
        uint32_t kraft = 0;
        for (int l = 1; l <= limit; l++) kraft += cnt[l] << (limit - l);
        while (kraft > (1u << limit)) {
            int l = limit - 1;
            while (!cnt[l]) l--;
            cnt[l]--;
            cnt[limit]--;
            cnt[l + 1] += 2;
            kraft--;
        }
        std::vector<RustUnstableSort::Pair> order(n);
        for (int i = 0; i < n; i++) order[i] = {(uint16_t)i, freq[i]};
        RustUnstableSort::sort(order.data(), order.size());
        int l = limit;
        for (const auto& o : order) {
            if (!o.f) continue;
            while (!cnt[l]) l--;
            len[o.sym] = (uint8_t)l;
            cnt[l]--;
        }
    }
    uint32_t next = 0;  // canonical codes, stored bit-reversed (LSB-first stream)
    for (int l = 1; l <= limit; l++) {
        for (int i = 0; i < n; i++) {
            if (len[i] != l) continue;
            uint32_t r = 0;
            for (int b = 0; b < l; b++) r |= ((next >> b) & 1u) << (l - 1 - b);
            code[i] = (uint16_t)r;
            next++;
        }
        next <<= 1;
    }
    return true;
}

// write_huffman_tree (:289-364)
void put_huffman_code(BitSink& w, const uint32_t* freq, int n, uint8_t* len, uint16_t* code)
{
    if (!huffman_lengths_codes(freq, n, len, code, 15)) {
        int sym = 0;
        while (sym < n && !freq[sym]) sym++;
        put_single_symbol_code(w, (unsigned)(uint8_t)(sym == n ? 0 : sym));
        return;
    }
    uint32_t clf[16] = {0};
    for (int i = 0; i < n; i++) clf[len[i]]++;
    uint8_t cll[16];
    uint16_t clc[16];
    const bool one_length = !huffman_lengths_codes(clf, 16, cll, clc, 7);
    static const int kOrder[19] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    w.put(0, 1);
    w.put(15, 4);
    for (int k = 0; k < 19; k++) {
        const int i = kOrder[k];
        w.put(i > 15 || !clf[i] ? 0 : (one_length ? 1 : cll[i]), 3);
    }
    if (n == 256) {
        w.put(1, 1);
        w.put(3, 3);
        w.put(254, 8);
    } else {
        w.put(0, 1);
    }
    if (!one_length)
        for (int i = 0; i < n; i++) w.put(clc[len[i]], cll[len[i]]);
}

// length_to_symbol (:355-362) for runs 5..4096
inline void run_symbol(uint32_t run, uint32_t& sym, uint32_t& extra)
{
    const uint32_t v = run - 1, hb = 31 - (uint32_t)__builtin_clz(v);
    extra = hb - 1;
    sym = 2 * hb + ((v >> (hb - 1)) & 1u);
}

}  // namespace

namespace {
// Per-pixel residual element: the packed ARGB residual (bytes r, g, b, a), or,
// for L8 images (the ALPH plane), only the green byte -- red and blue are 0
// and alpha constant there, so two residuals are equal exactly when their
// green bytes are.
template <class T> struct Px;
template <> struct Px<uint32_t> {
    static uint32_t g(uint32_t c) { return (c >> 8) & 255; }
    static uint32_t r(uint32_t c) { return c & 255; }
    static uint32_t b(uint32_t c) { return (c >> 16) & 255; }
    static uint32_t a(uint32_t c) { return c >> 24; }
};
template <> struct Px<uint8_t> {
    static uint32_t g(uint8_t c) { return c; }
    static uint32_t r(uint8_t) { return 0; }
    static uint32_t b(uint8_t) { return 0; }
    static uint32_t a(uint8_t) { return 0; }
};
// count_run (:366-393): repeats of px[p] after it, at most 4096
inline uint32_t run_after(const uint32_t* px, size_t p, size_t npx)
{
    const uint32_t c = px[p];
    uint32_t run = 0;
    while (run < 4096 && p + 1 + run < npx && px[p + 1 + run] == c) run++;
    return run;
}
inline uint32_t run_after(const uint8_t* px, size_t p, size_t npx)
{
    const uint8_t c = px[p];
    const size_t lim = std::min<size_t>(4096, npx - 1 - p);
    const uint64_t rep = 0x0101010101010101ull * c;
    size_t run = 0;
    while (run + 8 <= lim) {  // eight pixels per compare
        uint64_t v;
        memcpy(&v, px + p + 1 + run, 8);
        if (v != rep) {
            run += (size_t)__builtin_ctzll(v ^ rep) >> 3;
            return (uint32_t)run;
        }
        run += 8;
    }
    while (run < lim && px[p + 1 + run] == c) run++;
    return (uint32_t)run;
}

// The Huffman codes and the pixel/run symbols of encode_frame_lossless
// (:1040-1173) over the residuals px.
template <class T>
void code_pixels(const T* px, size_t npx, bool rgb, bool alpha, bool predictor, BitSink& w)
{
    using X = Px<T>;
    // symbol statistics: every pixel codes green (+ red/blue/alpha), then an
    // optional run of up to 4096 repeats of that pixel
    uint32_t fr[256] = {0}, fg[280] = {0}, fb[256] = {0}, fa[256] = {0};
    if (!rgb) fr[0] = fb[0] = 1;
    if (!alpha) fa[0] = 1;
    std::vector<uint16_t> runs;  // run after each coded pixel
    runs.reserve(npx / 64 + 16);
    for (size_t p = 0; p < npx;) {
        const T c = px[p];
        fg[X::g(c)]++;
        if (rgb) {
            fr[X::r(c)]++;
            fb[X::b(c)]++;
        }
        if (alpha) fa[X::a(c)]++;
        const uint32_t run = run_after(px, p, npx);
        if (run) {
            if (run <= 4) {
                fg[256 + run - 1]++;
            } else {
                uint32_t s, e;
                run_symbol(run, s, e);
                fg[256 + s]++;
            }
        }
        runs.push_back((uint16_t)run);
        p += 1 + run;
    }
    uint8_t lr[256], lg[280], lb[256], la[256];
    uint16_t cr[256], cg[280], cb[256], ca[256];
    memset(lr, 0, sizeof lr);
    memset(lb, 0, sizeof lb);
    memset(la, 0, sizeof la);
    memset(cr, 0, sizeof cr);
    memset(cb, 0, sizeof cb);
    memset(ca, 0, sizeof ca);
    put_huffman_code(w, fg, 280, lg, cg);
    if (rgb) {
        put_huffman_code(w, fr, 256, lr, cr);
        put_huffman_code(w, fb, 256, lb, cb);
    } else {
        put_single_symbol_code(w, 0);
        put_single_symbol_code(w, 0);
    }
    if (alpha) put_huffman_code(w, fa, 256, la, ca);
    else put_single_symbol_code(w, predictor ? 0 : 255);
    put_single_symbol_code(w, 1);  // distance code (unused)

    size_t k = 0;
    for (size_t p = 0; p < npx; k++) {
        const T c = px[p];
        const uint32_t g = X::g(c), r = X::r(c), b = X::b(c), a = X::a(c);
        uint64_t bits = cg[g];
        unsigned nb = lg[g];
        if (rgb) {
            bits |= (uint64_t)cr[r] << nb;
            nb += lr[r];
            bits |= (uint64_t)cb[b] << nb;
            nb += lb[b];
        }
        if (alpha) {
            bits |= (uint64_t)ca[a] << nb;
            nb += la[a];
        }
        w.put(bits, nb);
        const uint32_t run = runs[k];
        if (run) {
            if (run <= 4) {
                w.put(cg[256 + run - 1], lg[256 + run - 1]);
            } else {
                uint32_t s, e;
                run_symbol(run, s, e);
                w.put(cg[256 + s], lg[256 + s]);
                w.put((uint64_t)(run - 1) & ((1ull << e) - 1), e);
            }
        }
        p += 1 + run;
    }
    w.finish();
}

void put_transforms(BitSink& w, uint32_t width, uint32_t height, bool alpha, bool predictor, bool implicit_dims)
{
    if (!implicit_dims) {
        w.put(0x2f, 8);
        w.put(width - 1, 14);
        w.put(height - 1, 14);
        w.put(alpha ? 1 : 0, 1);
        w.put(0, 3);
    }
    w.put(5, 3);  // subtract-green transform
    if (predictor) {
        w.put(0x39, 6);  // predictor transform, size bits, no colour cache, mode-2 sub-image
        w.put(0, 1);
        put_single_symbol_code(w, 2);
        for (int i = 0; i < 4; i++) put_single_symbol_code(w, 0);
    }
    w.put(0, 1);  // no more transforms
    w.put(0, 1);  // no colour cache
    w.put(0, 1);  // no meta Huffman codes
}

// An L8 image read from byte `off` of every `bpp`-byte pixel (the grey plane,
// or the alpha channel of an LA8 / RGBA8 image for ALPH): its green residuals
// in one pass (subtract-green leaves green; the predictor takes the pixel above,
// on row 0 the pixel to the left, and 0 for the first pixel).
void l8_residuals(const uint8_t* data, int bpp, int off, uint32_t width, uint32_t height, bool predictor,
                  uint8_t* g)
{
    const size_t W = width;
    const uint8_t* s = data + off;
    if (!predictor) {
        for (size_t i = 0; i < W * height; i++) g[i] = s[i * bpp];
        return;
    }
    g[0] = s[0];
    for (size_t x = 1; x < W; x++) g[x] = (uint8_t)(s[x * bpp] - s[(x - 1) * bpp]);
    for (size_t y = 1; y < height; y++) {
        const uint8_t* cur = s + y * W * bpp;
        const uint8_t* up = cur - W * bpp;
        uint8_t* o = g + y * W;
        if (bpp == 1) {
            for (size_t x = 0; x < W; x++) o[x] = (uint8_t)(cur[x] - up[x]);
        } else {
            for (size_t x = 0; x < W; x++) o[x] = (uint8_t)(cur[x * bpp] - up[x * bpp]);
        }
    }
}
}  // namespace

// encode_frame_lossless (:945-1173) into `out` (appended).
int zw_vp8l_encode(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color, bool predictor,
                   bool implicit_dims, std::vector<uint8_t>& out)
{
    if (color < ZW_COLOR_L8 || color > ZW_COLOR_RGBA8) return ZW_EINVAL;
    const int bpp = color + 1;
    const bool rgb = color >= ZW_COLOR_RGB8, alpha = color == ZW_COLOR_LA8 || color == ZW_COLOR_RGBA8;
    if (!data && len) return ZW_EINVAL;
    if ((uint64_t)width * height * (uint64_t)bpp != (uint64_t)len) return ZW_EINVALID_BUFFER_SIZE;
    if (width == 0 || width > 16384 || height == 0 || height > 16384) return ZW_EINVALID_DIMENSIONS;
    BitSink w(out);
    put_transforms(w, width, height, alpha, predictor, implicit_dims);
    const size_t npx = (size_t)width * height;
    if (color == ZW_COLOR_L8) {
        std::vector<uint8_t> g(npx);
        l8_residuals(data, 1, 0, width, height, predictor, g.data());
        code_pixels(g.data(), npx, false, false, predictor, w);
        return ZW_OK;
    }

    // ARGB residuals, one uint32 per pixel (bytes r, g, b, a): expand, subtract
    // green, then the predictor's "pixel minus the pixel above (row 0: left)"
    std::vector<uint32_t> px(npx);
    auto pack = [](uint32_t r, uint32_t g, uint32_t b, uint32_t a) { return r | (g << 8) | (b << 16) | (a << 24); };
    parallel_for((int)height, [&](int y) {
        for (size_t x = 0; x < width; x++) {
            const size_t i = (size_t)y * width + x;
            const uint8_t* s = data + i * bpp;
            uint32_t r, g, b, a;
            switch (color) {
            case ZW_COLOR_LA8: r = g = b = s[0]; a = s[1]; break;
            case ZW_COLOR_RGB8: r = s[0]; g = s[1]; b = s[2]; a = 255; break;
            default: r = s[0]; g = s[1]; b = s[2]; a = s[3]; break;
            }
            px[i] = pack((r - g) & 255, g, (b - g) & 255, a);
        }
    });
    auto bytesub = [](uint32_t c, uint32_t p) {  // per-byte wrapping subtraction
        return ((c | 0x80808080u) - (p & 0x7f7f7f7fu)) ^ ((c ^ ~p) & 0x80808080u);
    };
    if (predictor) {
        std::vector<uint32_t> up(px);  // rows are differenced against the ORIGINAL row above
        parallel_for((int)height - 1, [&](int yy) {
            const size_t y = (size_t)yy + 1;
            for (size_t x = 0; x < width; x++) px[y * width + x] = bytesub(up[y * width + x], up[(y - 1) * width + x]);
        });
        for (size_t x = width - 1; x >= 1; x--) px[x] = bytesub(up[x], up[x - 1]);
        px[0] = bytesub(up[0], pack(0, 0, 0, 255));
    }
    code_pixels(px.data(), npx, rgb, alpha, predictor, w);
    return ZW_OK;
}

// encode_alpha_lossless (:1175-1222): the alpha channel as an L8 image with the
// predictor on and implicit dimensions, behind a one-byte header.
int zw_alph_encode(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                   std::vector<uint8_t>& out)
{
    if (color != ZW_COLOR_LA8 && color != ZW_COLOR_RGBA8) return ZW_EINVAL;
    if (width == 0 || width > 16384 || height == 0 || height > 16384) return ZW_EINVALID_DIMENSIONS;
    const int bpp = color == ZW_COLOR_LA8 ? 2 : 4;
    const size_t npx = (size_t)width * height;
    if (!data || len != npx * bpp) return ZW_EINVALID_BUFFER_SIZE;
    out.push_back(1);  // no preprocessing, no filtering, lossless compression
    std::vector<uint8_t> g(npx);
    l8_residuals(data, bpp, bpp - 1, width, height, true, g.data());
    BitSink w(out);
    put_transforms(w, width, height, false, true, true);
    code_pixels(g.data(), npx, false, false, true, w);
    return ZW_OK;
}

static int to_bytes(const std::vector<uint8_t>& v, zw_bytes* out)
{
    out->data = (uint8_t*)malloc(v.size() ? v.size() : 1);
    if (!out->data) return ZW_ENOMEM;
    memcpy(out->data, v.data(), v.size());
    out->len = v.size();
    return ZW_OK;
}

extern "C" int zw_encode_frame_lossless(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                                        int use_predictor, zw_bytes* out)
{
    if (!out) return ZW_EINVAL;
    out->data = nullptr;
    out->len = 0;
    std::vector<uint8_t> v;
    if (int r = zw_vp8l_encode(data, len, width, height, color, use_predictor != 0, false, v)) return r;
    return to_bytes(v, out);
}

extern "C" int zw_encode_alpha(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                               zw_bytes* out)
{
    if (!out) return ZW_EINVAL;
    out->data = nullptr;
    out->len = 0;
    std::vector<uint8_t> v;
    if (int r = zw_alph_encode(data, len, width, height, color, v)) return r;
    return to_bytes(v, out);
}

namespace {
void put_le32(std::vector<uint8_t>& o, uint32_t v)
{
    for (int i = 0; i < 4; i++) o.push_back((uint8_t)(v >> (8 * i)));
}
uint32_t chunk_bytes(size_t payload) { return (uint32_t)(payload + (payload & 1) + 8); }  // chunk_size (:1224)
void put_chunk(std::vector<uint8_t>& o, const char* tag, const uint8_t* p, size_t n)  // write_chunk (:1232)
{
    o.insert(o.end(), tag, tag + 4);
    put_le32(o, (uint32_t)n);
    if (n) o.insert(o.end(), p, p + n);
    if (n & 1) o.push_back(0);
}
}  // namespace

// The RIFF container of WebPEncoder::encode (:1317-1395): the simple form
// ("VP8 " / "VP8L" chunk only) without metadata and ALPH, else VP8X with
// ICCP, ALPH, the frame, EXIF and XMP in that order.  alph: the ALPH payload
// of a lossy encode with alpha, else null.
void zw_webp_wrap(std::vector<uint8_t>& o, const uint8_t* frame, size_t flen, const char* tag,
                  const std::vector<uint8_t>* alph, bool has_alpha, uint32_t width, uint32_t height,
                  const zw_metadata& md)
{
    const bool simple = !md.icc_len && !md.exif_len && !md.xmp_len && !alph;
    o.reserve(o.size() + flen + (alph ? alph->size() : 0) + md.icc_len + md.exif_len + md.xmp_len + 96);
    if (simple) {
        o.insert(o.end(), {'R', 'I', 'F', 'F'});
        put_le32(o, chunk_bytes(flen) + 4);
        o.insert(o.end(), {'W', 'E', 'B', 'P'});
        put_chunk(o, tag, frame, flen);
        return;
    }
    uint32_t total = 22 + chunk_bytes(flen);
    if (md.icc_len) total += chunk_bytes(md.icc_len);
    if (md.exif_len) total += chunk_bytes(md.exif_len);
    if (md.xmp_len) total += chunk_bytes(md.xmp_len);
    if (alph) total += chunk_bytes(alph->size());
    uint8_t flags = 0;
    if (md.xmp_len) flags |= 1 << 2;
    if (md.exif_len) flags |= 1 << 3;
    if (has_alpha) flags |= 1 << 4;
    if (md.icc_len) flags |= 1 << 5;
    o.insert(o.end(), {'R', 'I', 'F', 'F'});
    put_le32(o, total);
    o.insert(o.end(), {'W', 'E', 'B', 'P'});
    uint8_t x[10] = {flags, 0, 0, 0};
    for (int i = 0; i < 3; i++) {
        x[4 + i] = (uint8_t)((width - 1) >> (8 * i));
        x[7 + i] = (uint8_t)((height - 1) >> (8 * i));
    }
    put_chunk(o, "VP8X", x, 10);
    if (md.icc_len) put_chunk(o, "ICCP", md.icc, md.icc_len);
    if (alph) put_chunk(o, "ALPH", alph->data(), alph->size());
    put_chunk(o, tag, frame, flen);
    if (md.exif_len) put_chunk(o, "EXIF", md.exif, md.exif_len);
    if (md.xmp_len) put_chunk(o, "XMP ", md.xmp, md.xmp_len);
}

// WebPEncoder::encode (:1291-1398) with EncoderParams and metadata.
extern "C" int zw_encode_webp_ex(zw_ctx* ctx, const uint8_t* data, size_t len, uint32_t width, uint32_t height,
                                 int color, const zw_encoder_params* params, const zw_metadata* meta, zw_bytes* out)
{
    if (!out) return ZW_EINVAL;
    out->data = nullptr;
    out->len = 0;
    zw_encoder_params prm = {0, 95, 4, 1};  // EncoderParams::default(): lossless, predictor on
    if (params) prm = *params;
    zw_metadata md = {nullptr, 0, nullptr, 0, nullptr, 0};
    if (meta) md = *meta;
    if ((!md.icc && md.icc_len) || (!md.exif && md.exif_len) || (!md.xmp && md.xmp_len)) return ZW_EINVAL;
    if (color < ZW_COLOR_L8 || color > ZW_COLOR_RGBA8) return ZW_EINVAL;
    const bool has_alpha = color == ZW_COLOR_LA8 || color == ZW_COLOR_RGBA8;
    const bool lossy_alpha = prm.use_lossy && has_alpha;

    std::vector<uint8_t> frame;
    const char* tag;
    if (prm.use_lossy) {
        if (!ctx) return ZW_EINVAL;
        zw_bytes f = {nullptr, 0};
        if (int r = zw_encode_frame_lossy(ctx, data, len, width, height, color, prm.lossy_quality, prm.method, &f))
            return r;
        frame.assign(f.data, f.data + f.len);
        zw_bytes_free(&f);
        tag = "VP8 ";
    } else {
        if (int r = zw_vp8l_encode(data, len, width, height, color, prm.use_predictor_transform != 0, false, frame))
            return r;
        tag = "VP8L";
    }
    std::vector<uint8_t> alph;
    if (lossy_alpha)
        if (int r = zw_alph_encode(data, len, width, height, color, alph)) return r;
    std::vector<uint8_t> o;
    zw_webp_wrap(o, frame.data(), frame.size(), tag, lossy_alpha ? &alph : nullptr, has_alpha, width, height, md);
    return to_bytes(o, out);
}

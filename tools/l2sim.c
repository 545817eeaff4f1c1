// Trace-driven model of k_num2's B gathers in the eight 4 MB L2s (128-B lines,
// 16-way LRU), round 6: which unit order / placement would keep B in L2.
// Inputs: rp.bin (int64 row pointer) and col.bin (int32 columns) of A = B,
// e.g. K3' written by
//   python -c "import sys; sys.path.insert(0,'ia-spgemm_amd'); import ias; \
//     A = ias.gen_rmat(20, 20, .45, .15, .15, 2, 0); A.row_ptr.tofile('rp.bin'); A.col.tofile('col.bin')"
// Streaming rows = rows of > 256 products; `slots` waves in flight per XCD
// (6 workgroups of 4 waves x 32 CUs), each doing one step (256 products: a
// column line and a value line per product, unique lines per step = L2
// requests) per round.  usage: l2sim MODE [SLOTS] [S]
//   MODE 0: units of 64 entries in row order, workgroup b on XCD b % 8 (k_num2)
//   MODE 1: units cut at 8*S product-balanced B slices, XCD x takes slices [x*S, (x+1)*S)
//   MODE 2: the same slices, slice p on XCD p % 8, each XCD's queue by sweep p / 8
// Results and the measured A/B: profiles/r06/slices/, DESIGN.md §4g.
// gcc -O2 -o l2sim tools/l2sim.c
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#define NX 8
#define LINE 128
#define WAYS 16
static int SETS = 2048;  // 4 MB / 128 / 16

typedef struct { uint64_t tag[WAYS]; uint32_t age[WAYS]; } Set;
static Set *l2[NX];
static uint32_t clk[NX];
static uint64_t hits[NX], miss[NX];

static int access_line(int x, uint64_t line) {
    Set *s = &l2[x][line % SETS];
    uint64_t t = line + 1;
    int lru = 0;
    for (int w = 0; w < WAYS; ++w) {
        if (s->tag[w] == t) { s->age[w] = ++clk[x]; hits[x]++; return 1; }
        if (s->age[w] < s->age[lru]) lru = w;
    }
    s->tag[lru] = t; s->age[lru] = ++clk[x]; miss[x]++;
    return 0;
}

static int64_t *rp; static int32_t *col; static int64_t nrows, nent;
typedef struct { int32_t row, e0, e1; } Unit;

static int cmp_u64(const void *a, const void *b) { uint64_t x = *(uint64_t*)a, y = *(uint64_t*)b; return x < y ? -1 : x > y; }

// wave state
typedef struct { int64_t u; int32_t e; int32_t off; } Wave;  // current unit, current entry, offset within entry's B row

int main(int argc, char **argv) {
    int mode = atoi(argv[1]);
    int slots = argc > 2 ? atoi(argv[2]) : 768;   // waves in flight per XCD
    int nsl = argc > 3 ? atoi(argv[3]) : 1;       // time slices (mode 2)
    FILE *f = fopen("rp.bin", "rb"); fseek(f, 0, SEEK_END); nrows = ftell(f) / 8 - 1; fseek(f, 0, SEEK_SET);
    rp = malloc(8 * (nrows + 1)); fread(rp, 8, nrows + 1, f); fclose(f);
    nent = rp[nrows];
    col = malloc(4 * nent); f = fopen("col.bin", "rb"); fread(col, 4, nent, f); fclose(f);
    int64_t *blen = malloc(8 * nrows);
    for (int64_t i = 0; i < nrows; ++i) blen[i] = rp[i + 1] - rp[i];
    // streaming rows: products > 256
    int64_t nstream = 0, sprod = 0, sorted = 1;
    char *str = calloc(nrows, 1);
    double *wcol = calloc(nrows, sizeof(double));
    for (int64_t i = 0; i < nrows; ++i) {
        int64_t p = 0;
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) { p += blen[col[e]]; if (e > rp[i] && col[e] < col[e-1]) sorted = 0; }
        if (p > 256) { str[i] = 1; nstream++; sprod += p; for (int64_t e = rp[i]; e < rp[i + 1]; ++e) wcol[col[e]] += blen[col[e]]; }
    }
    fprintf(stderr, "rows %ld entries %ld stream rows %ld products %ld sorted %ld\n", nrows, nent, nstream, sprod, sorted);
    // column range boundaries for NX (or NX*nsl) parts of equal products
    int nparts = (mode == 0) ? 1 : NX * nsl;
    int32_t *bnd = malloc(sizeof(int32_t) * (nparts + 1));
    {
        double tot = 0; for (int64_t j = 0; j < nrows; ++j) tot += wcol[j];
        double acc = 0; int k = 1; bnd[0] = 0;
        for (int64_t j = 0; j < nrows && k < nparts; ++j) { acc += wcol[j]; while (k < nparts && acc >= tot * k / nparts) bnd[k++] = (int32_t)(j + 1); }
        while (k <= nparts) bnd[k++] = (int32_t)nrows;
        bnd[nparts] = (int32_t)nrows;
    }
    // build unit queues per XCD
    int64_t cap = nent + nrows * nparts + 16;
    Unit *q[NX]; int64_t qn[NX] = {0};
    for (int x = 0; x < NX; ++x) q[x] = malloc(sizeof(Unit) * (cap / NX * 2 + 1000000));
    int64_t gu = 0;  // global unit counter (mode 0: WG b = gu/4 -> XCD b%8)
    if (mode == 0) {
        for (int64_t i = 0; i < nrows; ++i) if (str[i]) {
            int32_t n = (int32_t)(rp[i + 1] - rp[i]);
            for (int32_t e0 = 0; e0 < n; e0 += 64) { int x = (int)((gu / 4) % NX); q[x][qn[x]++] = (Unit){(int32_t)i, e0, e0 + 64 < n ? e0 + 64 : n}; gu++; }
        }
    } else {
        // mode 1: part k*nsl+s ... XCD = part % NX? parts ordered by column: XCD x gets parts [x*nsl, (x+1)*nsl)
        // mode 2: time slices: part p -> XCD p % NX, slice p / NX; queue ordered by slice then row
        for (int sl = 0; sl < nsl; ++sl)
        for (int64_t i = 0; i < nrows; ++i) if (str[i]) {
            int64_t s0 = rp[i], n = rp[i + 1] - rp[i];
            for (int x = 0; x < NX; ++x) {
                int p = (mode == 1) ? x * nsl + sl : sl * NX + x;
                int32_t lo = bnd[p], hi = bnd[p + 1];
                // entries with col in [lo, hi)
                int64_t a = 0; while (a < n && col[s0 + a] < lo) ++a;
                int64_t b = a; while (b < n && col[s0 + b] < hi) ++b;
                for (int64_t e0 = a; e0 < b; e0 += 64) q[x][qn[x]++] = (Unit){(int32_t)i, (int32_t)e0, (int32_t)(e0 + 64 < b ? e0 + 64 : b)};
            }
        }
    }
    int64_t tu = 0; for (int x = 0; x < NX; ++x) tu += qn[x];
    fprintf(stderr, "units %ld (per xcd:", tu); for (int x = 0; x < NX; ++x) fprintf(stderr, " %ld", qn[x]); fprintf(stderr, ")\n");
    for (int x = 0; x < NX; ++x) l2[x] = calloc(SETS, sizeof(Set));
    // simulate: per XCD, `slots` waves; round robin, each wave does a step of 256 products
    Wave *w[NX]; int64_t nxt[NX];
    uint64_t *lines = malloc(8 * 1024);
    int64_t steps = 0, rounds = 0, lanes_used = 0;
    for (int x = 0; x < NX; ++x) { w[x] = malloc(sizeof(Wave) * slots); nxt[x] = 0; for (int s = 0; s < slots; ++s) w[x][s].u = -1; }
    int active = 1;
    while (active) {
        active = 0; rounds++;
        for (int x = 0; x < NX; ++x) for (int s = 0; s < slots; ++s) {
            Wave *v = &w[x][s];
            if (v->u < 0) { if (nxt[x] >= qn[x]) continue; v->u = nxt[x]++; v->e = q[x][v->u].e0; v->off = 0; }
            active = 1;
            Unit U = q[x][v->u];
            int64_t base = rp[U.row];
            int nl = 0, np = 0;
            while (np < 256 && v->e < U.e1) {
                int32_t j = col[base + v->e];
                int64_t bs = rp[j], bl = blen[j];
                while (np < 256 && v->off < bl) {
                    int64_t k = bs + v->off;
                    lines[nl++] = ((uint64_t)k * 4) / LINE;
                    lines[nl++] = (((uint64_t)k * 8) / LINE) + (1ull << 40);
                    ++np; ++v->off;
                }
                if (v->off >= bl) { v->e++; v->off = 0; }
            }
            steps++; lanes_used += np;
            qsort(lines, nl, 8, cmp_u64);
            for (int i = 0; i < nl; ++i) if (i == 0 || lines[i] != lines[i - 1]) access_line(x, lines[i]);
            if (v->e >= U.e1) v->u = -1;
        }
    }
    uint64_t H = 0, M = 0;
    for (int x = 0; x < NX; ++x) { H += hits[x]; M += miss[x]; }
    fprintf(stderr, "per xcd miss:"); for (int x = 0; x < NX; ++x) fprintf(stderr, " %.0fM", miss[x] / 1e6); fprintf(stderr, "\n");
    printf("mode %d slots %d nsl %d: steps %ld lane-util %.3f rounds %ld  hit %.3f  miss bytes %.2f GB  (gathered %.2f GB)\n",
           mode, slots, nsl, steps, lanes_used / (256.0 * steps), rounds, H / (double)(H + M), M * (double)LINE / 1e9, sprod * 12.0 / 1e9);
    return 0;
}

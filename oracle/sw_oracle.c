/*
 * Smith-Waterman CPU oracle — TEST INFRASTRUCTURE ONLY (see sw_oracle.h).
 *
 * The reference sweeps anti-diagonals with AVX2 (PairWiseSW.h:100-228); every
 * cell depends only on its left, upper and upper-left neighbours and the
 * arithmetic is int32, so this restatement sweeps plain rows and gets the same
 * values. Paths below are relative to src/haplotypecaller/smithwaterman/.
 */
#include "sw_oracle.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum {   /* native/smithwaterman_common.h:21-29 */
    OP_MATCH = 0, OP_INSERT = 1, OP_DELETE = 2, INSERT_EXT = 4, DELETE_EXT = 8,
    OVH_SOFTCLIP = 9, OVH_INDEL = 10, OVH_LEADING_INDEL = 11, OVH_IGNORE = 12
};
#define MIN_CUTOFF (-100000000)   /* MATRIX_MIN_CUTOFF, :50 */
#define LOW_INIT (INT_MIN / 2)    /* LOW_INIT_VALUE, :51 */

static int imax(int a, int b) { return a > b ? a : b; }
static int iabs(int a) { return a < 0 ? -a : a; }

/* H(0, x) and H(x, 0) for x >= 1: the boundary writes after each anti-diagonal
 * (PairWiseSW.h:188-197); H(0, 0) = 0 (:80). */
static int boundary(int overhang, int open, int extend, int x)
{
    return (overhang == OVH_INDEL || overhang == OVH_LEADING_INDEL) ? open + (x - 1) * extend : 0;
}

/* Run-length CIGAR under construction, in traceback order (end to start). */
typedef struct {
    int* op;
    int* len;
    int n;
} Elems;

static void push(Elems* e, int op, int len)
{
    e->op[e->n] = op;
    e->len[e->n] = len;
    ++e->n;
}

int hco_sw_align(int match, int mismatch, int open, int extend,
                 const uint8_t* s1, int n1, const uint8_t* s2, int n2,
                 int overhang, char* cigar, int cap, int* score)
{
    const int W = n2 + 1;
    const size_t cells = (size_t)(n1 + 1) * (size_t)W;
    int* H = (int*)malloc(sizeof(int) * cells);
    int* E = (int*)malloc(sizeof(int) * cells);
    int* F = (int*)malloc(sizeof(int) * cells);
    uint8_t* bt = (uint8_t*)malloc(cells);
    Elems el = {(int*)malloc(sizeof(int) * (size_t)(n1 + n2 + 4)),
                (int*)malloc(sizeof(int) * (size_t)(n1 + n2 + 4)), 0};

    H[0] = 0;
    for (int j = 1; j <= n2; ++j) {
        H[j] = boundary(overhang, open, extend, j);
        F[j] = LOW_INIT;   /* F[jhi] = lowInitValue, :198 */
    }
    for (int i = 1; i <= n1; ++i) {
        H[(size_t)i * W] = boundary(overhang, open, extend, i);
        E[(size_t)i * W] = LOW_INIT;   /* E[MAX_SEQ_LEN - ilo] = lowInitValue, :199 */
    }
    /* MAIN_CODE (PairWiseSW.h:4-38), one cell at a time. */
    for (int i = 1; i <= n1; ++i) {
        const size_t r = (size_t)i * W, u = (size_t)(i - 1) * W;
        for (int j = 1; j <= n2; ++j) {
            const int eo = H[r + j - 1] + open, ee = E[r + j - 1] + extend;
            const int e = imax(eo, ee);
            const int fo = H[u + j] + open, fe = F[u + j] + extend;
            const int f = imax(fe, fo);
            int h = imax(MIN_CUTOFF, H[u + j - 1] + (s1[i - 1] == s2[j - 1] ? match : mismatch));
            int b = e > h ? OP_INSERT : OP_MATCH;
            h = imax(h, e);
            if (f > h) b = OP_DELETE;
            h = imax(h, f);
            b |= (eo > ee ? 0 : INSERT_EXT) | (fo > fe ? 0 : DELETE_EXT);
            E[r + j] = e;
            F[r + j] = f;
            H[r + j] = h;
            bt[r + j] = (uint8_t)b;
        }
    }
    /* End point: last row (SOFTCLIP / IGNORE only), then last column, in
     * anti-diagonal order with the reference's tie-breaks (:201-226). */
    int best = INT_MIN, bi = 0, bj = 0;
    for (int d = 1; d <= n1 + n2; ++d) {
        if (d >= n1 + 1 && (overhang == OVH_SOFTCLIP || overhang == OVH_IGNORE)) {
            const int j = d - n1, sc = H[(size_t)n1 * W + j];
            if (best < sc || (best == sc && iabs(n1 - j) < iabs(bi - bj))) {
                best = sc;
                bi = n1;
                bj = j;
            }
        }
        if (d >= n2 + 1) {
            const int i = d - n2, sc = H[(size_t)i * W + n2];
            if (best < sc || (best == sc && (bj == n2 || iabs(i - n2) <= iabs(bi - bj)))) {
                best = sc;
                bi = i;
                bj = n2;
            }
        }
    }
    if (score) *score = best;

    /* Traceback (getCIGAR, :254-366). */
    int i = bi, j = bj;
    if (overhang == OVH_INDEL) {
        i = n1;
        j = n2;
    } else if (overhang == OVH_LEADING_INDEL) {
        j = n2;
    }
    if (j < n2) push(&el, OVH_SOFTCLIP, n2 - j);
    int state = 0;
    while (i > 0 && j > 0) {
        const int b = bt[(size_t)i * W + j];
        if (state == INSERT_EXT) {
            --j;
            ++el.len[el.n - 1];
            state = b & INSERT_EXT;
        } else if (state == DELETE_EXT) {
            --i;
            ++el.len[el.n - 1];
            state = b & DELETE_EXT;
        } else if ((b & 3) == OP_MATCH) {
            --i;
            --j;
            push(&el, OP_MATCH, 1);
            state = 0;
        } else if ((b & 3) == OP_INSERT) {
            --j;
            push(&el, OP_INSERT, 1);
            state = b & INSERT_EXT;
        } else {
            --i;
            push(&el, OP_DELETE, 1);
            state = b & DELETE_EXT;
        }
    }
    int offset;
    if (overhang == OVH_SOFTCLIP) {
        if (j > 0) push(&el, OVH_SOFTCLIP, j);
        offset = i;
    } else if (overhang == OVH_IGNORE) {
        if (j > 0 && el.n > 0) push(&el, el.op[el.n - 1], j);
        offset = i - j;
    } else {
        if (i > 0) push(&el, OP_DELETE, i);
        else if (j > 0) push(&el, OP_INSERT, j);
        offset = 0;
    }
    /* Merge equal neighbours (:368-386) and print from the start (:388-413). */
    int m = 0;
    for (int k = 1; k < el.n; ++k) {
        if (el.op[k] == el.op[m]) {
            el.len[m] += el.len[k];
        } else {
            ++m;
            el.op[m] = el.op[k];
            el.len[m] = el.len[k];
        }
    }
    const int count = el.n ? m + 1 : 0;
    int pos = 0;
    for (int k = count - 1; k >= 0 && pos >= 0; --k) {
        const char c = el.op[k] == OP_MATCH ? 'M' : el.op[k] == OP_INSERT ? 'I'
                     : el.op[k] == OP_DELETE ? 'D' : el.op[k] == OVH_SOFTCLIP ? 'S' : 'R';
        const int w = snprintf(cigar + pos, (size_t)(cap - pos), "%d%c", el.len[k], c);
        pos = (w < 0 || pos + w >= cap) ? -1 : pos + w;
    }
    if (pos >= 0 && count == 0) cigar[0] = 0;
    free(H);
    free(E);
    free(F);
    free(bt);
    free(el.op);
    free(el.len);
    return pos < 0 ? INT_MIN : offset;
}

int hco_sw_is_all_match(const uint8_t* ref, int ref_len, const uint8_t* alt, int alt_len)
{
    if (ref_len != alt_len) return 0;
    int mismatch = 0;
    for (int i = 0; mismatch <= 2 && i < ref_len; ++i) mismatch += ref[i] != alt[i];
    return mismatch <= 2;
}

int hco_sw_batch(long n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                 const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts,
                 int match, int mismatch, int open, int extend, int overhang, int shortcut,
                 int32_t* offsets, char* cigars, int stride, int nthreads)
{
    int bad = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : bad)
#endif
    for (long k = 0; k < n; ++k) {
        const uint8_t* r = refs + ref_off[k];
        const uint8_t* a = alts + alt_off[k];
        char* out = cigars + (size_t)k * (size_t)stride;
        if (shortcut && hco_sw_is_all_match(r, ref_len[k], a, alt_len[k])) {
            offsets[k] = 0;   /* {0, Cigar(1, {ref.size(), M})}, intel_smithwaterman.hpp:36-37 */
            bad |= snprintf(out, (size_t)stride, "%dM", ref_len[k]) >= stride;
            continue;
        }
        offsets[k] = hco_sw_align(match, mismatch, open, extend, r, ref_len[k], a, alt_len[k], overhang,
                                  out, stride, NULL);
        bad |= offsets[k] == INT_MIN;
    }
    (void)nthreads;
    return bad ? -1 : 0;
}

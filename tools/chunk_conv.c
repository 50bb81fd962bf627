/* Do speculative chunk starts converge for a huge object's AET?  (CPU
 * experiment for DESIGN §4.4, driven by tools/chunk_conv.py.)
 *
 * Input (stdin, binary): int32 n, H, then n records {float X, G; int32 Left,
 * YMin, YMax} in FillEdgeTable + MergeSort order (one object).  The list
 * dynamics restate oracle/prk_oracle.c or_aet_walk (projekt.cpp:3654-3869)
 * on the keys only: insertion before the first entry the new edge sorts
 * before, expiry of YMax <= Row, pairs stepped (X += G) and their two swaps.
 *
 * For every chunk start r0 (multiple of C) it starts a walk at row r0 - W
 * from the sorted list of the edges active there (true X values) and checks
 * whether the list at the start of row r0 equals the true walk's.
 * Output: per (C, W): chunks, chunks whose start differs, odd rows. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float X, G; int Left, YMin, YMax; } Edge;

static int before(const Edge *a, const Edge *b)
{
    return a->X < b->X || (a->X == b->X && (a->G < b->G || (a->G == b->G && a->Left < b->Left)));
}

static int n, H, FirstRow, MaxY;
static Edge *E;
static int *rowStart; /* edges with YMin == r: [rowStart[r], rowStart[r+1]) (sorted by YMin) */

/* One row of the walk on list L (ids, length *m) with edge state X[];
 * returns 1 if the row had an odd entry count. */
static int walk_row(int Row, int *L, int *m, float *X)
{
    int k = *m;
    for (int i = rowStart[Row - FirstRow]; i < rowStart[Row - FirstRow + 1]; ++i) {
        Edge c = E[i];
        c.X = X[i];
        int pos = k;
        for (int j = 0; j < k; ++j) {
            Edge o = E[L[j]];
            o.X = X[L[j]];
            if (before(&c, &o)) { pos = j; break; }
        }
        memmove(L + pos + 1, L + pos, (size_t)(k - pos) * sizeof(int));
        L[pos] = i;
        ++k;
    }
    int w = 0;
    for (int j = 0; j < k; ++j)
        if (E[L[j]].YMax > Row) L[w++] = L[j];
    k = w;
    *m = k;
    /* pairing: positions of pair (2p, 2p+1) in the current list */
    int odd = k & 1;
    for (int p = 0; 2 * p + 1 < k; ++p) {
        int a = 2 * p, b = 2 * p + 1;
        X[L[a]] += E[L[a]].G;
        X[L[b]] += E[L[b]].G;
        if (X[L[a]] > X[L[b]]) { int t = L[a]; L[a] = L[b]; L[b] = t; }
        if (p > 0 && X[L[a - 1]] > X[L[a]]) { int t = L[a - 1]; L[a - 1] = L[a]; L[a] = t; }
    }
    return odd;
}


int main(int argc, char **argv)
{
    if (fread(&n, 4, 1, stdin) != 1 || fread(&H, 4, 1, stdin) != 1) return 1;
    E = malloc(sizeof(Edge) * (size_t)n);
    if (fread(E, sizeof(Edge), (size_t)n, stdin) != (size_t)n) return 1;
    FirstRow = E[0].YMin;
    int MaxRow = E[0].YMax;
    for (int i = 1; i < n; ++i) if (E[i].YMax > MaxRow) MaxRow = E[i].YMax;
    MaxY = MaxRow < H ? MaxRow : H;
    int rows = MaxY - FirstRow;
    rowStart = calloc((size_t)rows + 2, sizeof(int));
    { int i = 0; for (int r = 0; r <= rows; ++r) { while (i < n && E[i].YMin < FirstRow + r) ++i; rowStart[r] = i; } rowStart[rows + 1] = n; }
    /* (edges with YMin >= MaxY are never inserted) */
    int Cs[] = {8, 16, 32}, Ws[] = {0, 4, 8, 16, 32};
    int *L = malloc(sizeof(int) * (size_t)n), *L2 = malloc(sizeof(int) * (size_t)n);
    float *X = malloc(sizeof(float) * (size_t)n), *X2 = malloc(sizeof(float) * (size_t)n);
    /* true walk: lists and X at every row start, kept for rows that are chunk starts of C = 8 */
    int nst = rows / 8 + 1;
    int **TL = calloc((size_t)nst, sizeof(int *)), *TM = calloc((size_t)nst, sizeof(int));
    float **TX = calloc((size_t)nst, sizeof(float *)); /* X of the listed edges, in list order */
    for (int i = 0; i < n; ++i) X[i] = E[i].X;
    int m = 0, odd_rows = 0, maxm = 0;
    for (int r = 0; r < rows; ++r) {
        if (r % 8 == 0) {
            TL[r / 8] = malloc(sizeof(int) * (size_t)(m + 1));
            memcpy(TL[r / 8], L, sizeof(int) * (size_t)m);
            TM[r / 8] = m;
            TX[r / 8] = malloc(sizeof(float) * (size_t)(m + 1));
            for (int j = 0; j < m; ++j) TX[r / 8][j] = X[L[j]];
        }
        odd_rows += walk_row(FirstRow + r, L, &m, X);
        if (m > maxm) maxm = m;
    }
    printf("edges %d rows %d odd rows %d most listed %d\n", n, rows, odd_rows, maxm);
    for (int ci = 0; ci < 3; ++ci)
        for (int wi = 0; wi < 5; ++wi) {
            int C = Cs[ci], W = Ws[wi];
            if (W % 8 || C % 8) continue;
            int chunks = 0, bad = 0;
            for (int r0 = C; r0 < rows; r0 += C) {
                int rs = r0 - W;
                if (rs < 0) rs = 0;
                /* sorted start at rs: the true list's entries, sorted by (X, G, Left), ties by edge order */
                int k = TM[rs / 8];
                memcpy(L2, TL[rs / 8], sizeof(int) * (size_t)k);
                for (int j = 0; j < k; ++j) X2[L2[j]] = TX[rs / 8][j];
                for (int i = rowStart[rs]; i < rowStart[r0 < rows ? r0 : rows]; ++i) X2[i] = E[i].X;
                /* insertion sort (stable) by the key at rs */
                for (int a = 1; a < k; ++a) {
                    int v = L2[a], b = a - 1;
                    Edge ev = E[v]; ev.X = X2[v];
                    while (b >= 0) {
                        Edge eb = E[L2[b]]; eb.X = X2[L2[b]];
                        if (before(&ev, &eb) || (!before(&eb, &ev) && v < L2[b])) { L2[b + 1] = L2[b]; --b; }
                        else break;
                    }
                    L2[b + 1] = v;
                }
                for (int r = rs; r < r0; ++r) walk_row(FirstRow + r, L2, &k, X2);
                ++chunks;
                if (k != TM[r0 / 8] || memcmp(L2, TL[r0 / 8], sizeof(int) * (size_t)k)) ++bad;
            }
            printf("C %2d W %2d: %d chunks, %d starts differ from the true list\n", C, W, chunks, bad);
            fflush(stdout);
        }
    return 0;
}

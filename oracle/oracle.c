/*
 * ORACLE — CPU restatement (test infrastructure only; see oracle.h).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off). pow() is always called
 * through a volatile function pointer so gcc cannot fold pow(x,2) into x*x;
 * glibc pow and x*x differ in ~0.08% of inputs (SURVEY.md §7 "Hard parts"),
 * and the reference (built at -O0) really calls pow.
 */
#include "oracle.h"

#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double (*volatile pow_fn)(double, double) = pow;
static double (*volatile sqrt_fn)(double) = sqrt;

/* assignment2.h:141-144 and :196 — identical expression, left-to-right. */
static double city_distance(const oracle_city *a, const oracle_city *b)
{
    double dx = pow_fn(a->x - b->x, 2);
    double dy = pow_fn(a->y - b->y, 2);
    return sqrt_fn(dx + dy);
}

void oracle_distance_matrix(const oracle_city *cities, int n, double *d)
{
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            d[i * n + j] = city_distance(&cities[i], &cities[j]);
}

/*
 * tsp.cpp:405-509 restated on a dense array G[S][k], S a bitmask over local
 * cities 1..N (bit k-1), k in S = last city:
 *   |S|==2   G[{i,k}][k] = d[i][k] + d[0][i]                    (tsp.cpp:424-438)
 *   |S|>=3   G[S][k] = min over m in S\{k}, ascending, strict <, starting from
 *            INT_MAX, of G[S\{k}][m] + d[m][k]                   (tsp.cpp:442-481)
 *            (the reference's s=2 pass never overwrites, tsp.cpp:478)
 *   closing  min over m ascending, strict <, from INT_MAX, of
 *            G[full][m] + d[m][0]                                (tsp.cpp:483-499)
 * The reference stores, per state, the path of its FIRST strict-minimum
 * predecessor; backtracking with "smallest m whose candidate equals the state
 * value" reproduces exactly that path.
 */
int oracle_solve_block(const double *d, int n, double *cost, int32_t *tour)
{
    if (n < 2)
        return -1;
    if (n == 2)
    {
        /* tsp.cpp:484-502 with cityNums={1}: key(empty,1) default-inserts cost 0. */
        *cost = 0.0 + d[1 * n + 0];
        tour[0] = 1;
        tour[1] = 0;
        return 2;
    }
    const int N = n - 1;
    const uint32_t full = (1u << N) - 1u;
    double *G = (double *)malloc(sizeof(double) * ((size_t)1 << N) * (size_t)N);
    if (!G)
        return -1;
#define GV(S, k) G[(size_t)(S) * (size_t)N + (size_t)((k)-1)]
    for (uint32_t S = 1; S <= full; S++)
    {
        int pc = __builtin_popcount(S);
        if (pc < 2)
            continue;
        for (int k = 1; k <= N; k++)
        {
            if (!(S & (1u << (k - 1))))
                continue;
            uint32_t T = S & ~(1u << (k - 1));
            if (pc == 2)
            {
                int i = __builtin_ctz(T) + 1;
                GV(S, k) = d[i * n + k] + d[0 * n + i];
                continue;
            }
            double best = (double)INT_MAX;
            for (int m = 1; m <= N; m++)
            {
                if (!(T & (1u << (m - 1))))
                    continue;
                double cur = GV(T, m) + d[m * n + k];
                if (cur < best)
                    best = cur;
            }
            GV(S, k) = best;
        }
    }
    double best = (double)INT_MAX;
    int bestM = -1;
    for (int m = 1; m <= N; m++)
    {
        double cur = GV(full, m) + d[m * n + 0];
        if (cur < best)
        {
            best = cur;
            bestM = m;
        }
    }
    if (bestM < 0)
    {
        free(G);
        return -1; /* reference: bestM uninitialised (UB) */
    }
    *cost = best;
    tour[0] = 0;
    tour[n] = 0;
    tour[n - 1] = bestM;
    uint32_t S = full;
    int k = bestM;
    int pos = n - 2;
    while (__builtin_popcount(S) > 2)
    {
        uint32_t T = S & ~(1u << (k - 1));
        int pick = -1;
        for (int m = 1; m <= N; m++)
        {
            if (!(T & (1u << (m - 1))))
                continue;
            if (GV(T, m) + d[m * n + k] == GV(S, k))
            {
                pick = m;
                break;
            }
        }
        if (pick < 0)
        {
            free(G);
            return -1;
        }
        tour[pos--] = pick;
        S = T;
        k = pick;
    }
    /* |S|==2: S={i,k}, stored path {0,i} (tsp.cpp:433). */
    tour[pos--] = __builtin_ctz(S & ~(1u << (k - 1))) + 1;
#undef GV
    free(G);
    return n + 1;
}

/* tsp.cpp:136-157; ISSQUARE from assignment2.h:11. */
void oracle_blocks_per_dim(int B, int *rows, int *cols)
{
    double r = sqrt((double)B);
    if (r - floor(r) == 0)
    {
        *rows = (int)r;
        *cols = (int)r;
        return;
    }
    int divisor = 2;
    while (B % divisor != 0)
        divisor++;
    *rows = divisor;
    *cols = B / divisor;
}

/* assignment2.h:86-91 */
static double f_rand(double lo, double hi)
{
    double f = (double)rand() / RAND_MAX;
    return lo + f * (hi - lo);
}

/* tsp.cpp:373-403. Spacing is float (tsp.cpp:378-379); row*spacing is a float
 * product promoted to double at the call. */
void oracle_generate(int n, int B, int X, int Y, oracle_city *out)
{
    int R, C;
    oracle_blocks_per_dim(B, &R, &C);
    srand(0);
    float xs = X / (float)R;
    float ys = Y / (float)C;
    int id = 0;
    for (int i = 0; i < R * C; i++)
    {
        for (int j = 0; j < n; j++)
        {
            int row = (i - (i % R)) / R;
            int col = (C - (i % C)) - 1;
            float x0 = row * xs, x1 = (row + 1) * xs;
            float y0 = col * ys, y1 = (col + 1) * ys;
            oracle_city c;
            c.id = id;
            c.x = f_rand(x0, x1);
            c.y = f_rand(y0, y1);
            out[(size_t)i * n + j] = c;
            id++;
        }
    }
}

/* tsp.cpp:167-171 */
void oracle_distribution_counts(int B, int P, int *cnt)
{
    for (int r = 0; r < P; r++)
        cnt[r] = 0;
    for (int left = B; left > 0; left--)
        cnt[left % P]++;
}

/* tsp.cpp:197-200: ((d(A,D) + d(B,C)) - d(A,B)) - d(C,D) */
static double swap_pair_cost(const oracle_city *a, const oracle_city *b, const oracle_city *c, const oracle_city *e)
{
    return city_distance(a, e) + city_distance(b, c) - city_distance(a, b) - city_distance(c, e);
}

/* tsp.cpp:202-269. Rotations are index arithmetic: at outer step i the pair is
 * (c1[i], c1[(i+1)%L1]), at inner step j (c2[j], c2[(j+1)%L2]). */
int oracle_merge_blocks(const oracle_city *p1, int L1, double c1, const oracle_city *p2, int L2, double c2,
                        oracle_city *out, double *cost)
{
    double best = (double)INT_MAX;
    int bi = 0, bj = 0;
    for (int i = 0; i < L1; i++)
        for (int j = 0; j < L2; j++)
        {
            double sc = swap_pair_cost(&p1[i], &p1[(i + 1) % L1], &p2[j], &p2[(j + 1) % L2]);
            if (sc < best)
            {
                best = sc;
                bi = i;
                bj = j;
            }
        }
    const int idA = p1[bi].id, idB = p1[(bi + 1) % L1].id, idC = p2[bj].id;
    /* cities2 without its last element, rotated left until [0].id == C.id, then once more */
    const int L2m = L2 - 1;
    int rot = 0;
    while (rot < L2m && p2[rot].id != idC)
        rot++;
    if (rot == L2m)
        return -1; /* the reference's while loop (tsp.cpp:236-239) never ends */
    rot = (rot + 1) % L2m;
    int o = 0;
    int flag = 1;
    for (int i = 0; i < L1; i++)
    {
        out[o++] = p1[i];
        if ((p1[i].id == idA || p1[i].id == idB) && flag)
        {
            flag = 0;
            for (int j = L2m - 1; j >= 0; j--)
                out[o++] = p2[(rot + j) % L2m];
        }
    }
    *cost = c1 + c2 + best;
    return o;
}

typedef struct
{
    oracle_city *p;
    int len, cap;
    double cost;
} sol_t;

static void sol_reserve(sol_t *s, int cap)
{
    if (s->cap < cap)
    {
        s->cap = cap * 2;
        s->p = (oracle_city *)realloc(s->p, sizeof(oracle_city) * (size_t)s->cap);
    }
}

static int sol_merge(sol_t *s1, const sol_t *s2)
{
    oracle_city *out = (oracle_city *)malloc(sizeof(oracle_city) * (size_t)(s1->len + s2->len));
    double cost;
    int L = oracle_merge_blocks(s1->p, s1->len, s1->cost, s2->p, s2->len, s2->cost, out, &cost);
    if (L < 0)
    {
        free(out);
        return -1;
    }
    free(s1->p);
    s1->p = out;
    s1->len = L;
    s1->cap = s1->len + s2->len;
    s1->cost = cost;
    return 0;
}

static void log_append(char *log, int logcap, int *used, const char *line)
{
    if (!log || logcap <= 0)
        return;
    int n = (int)strlen(line);
    if (*used + n >= logcap)
        n = logcap - 1 - *used;
    if (n > 0)
    {
        memcpy(log + *used, line, (size_t)n);
        *used += n;
    }
    log[*used] = 0;
}

/* Receive step of MPI_ManualReduce (tsp.cpp:87-98 / 109-120): the receiver's
 * function-local `path` (tsp.cpp:67) keeps growing; the block handed to
 * mergeBlocks carries the WHOLE accumulated path with the sender's cost. */
static int tree_receive(sol_t *recv_acc, sol_t *self, const sol_t *sender)
{
    sol_reserve(recv_acc, recv_acc->len + sender->len);
    memcpy(recv_acc->p + recv_acc->len, sender->p, sizeof(oracle_city) * (size_t)sender->len);
    recv_acc->len += sender->len;
    sol_t blk = {recv_acc->p, recv_acc->len, recv_acc->cap, sender->cost};
    return sol_merge(self, &blk);
}

int oracle_pipeline(int n, int B, int X, int Y, int P, double *final_cost, char *log, int logcap)
{
    if (log && logcap > 0)
        log[0] = 0;
    if (n < 2 || B < 1 || P < 1 || B < P)
        return -1;
    int used = 0;
    oracle_city *cities = (oracle_city *)malloc(sizeof(oracle_city) * (size_t)B * (size_t)n);
    oracle_generate(n, B, X, Y, cities);
    sol_t *blocks = (sol_t *)calloc((size_t)B, sizeof(sol_t));
    double *d = (double *)malloc(sizeof(double) * (size_t)n * (size_t)n);
    int32_t tour[64];
    for (int b = 0; b < B; b++)
    {
        const oracle_city *blk = cities + (size_t)b * n;
        oracle_distance_matrix(blk, n, d);
        int L = oracle_solve_block(d, n, &blocks[b].cost, tour);
        if (L < 0)
            return -1;
        blocks[b].p = (oracle_city *)malloc(sizeof(oracle_city) * (size_t)L);
        blocks[b].len = blocks[b].cap = L;
        for (int i = 0; i < L; i++)
            blocks[b].p[i] = blk[tour[i]]; /* convPathToCityPath, assignment2.h:76-84 */
    }
    free(d);
    free(cities);

    int rc = 0;
    int *cnt = (int *)malloc(sizeof(int) * (size_t)P);
    oracle_distribution_counts(B, P, cnt);
    sol_t *rank = (sol_t *)calloc((size_t)P, sizeof(sol_t));
    int next = 0;
    for (int r = 0; r < P; r++)
    {
        /* local fold, tsp.cpp:348-352 */
        rank[r] = blocks[next];
        blocks[next].p = NULL;
        next++;
        for (int j = 1; j < cnt[r]; j++, next++)
            if (sol_merge(&rank[r], &blocks[next]) < 0)
                rc = -1;
    }

    sol_t *acc = (sol_t *)calloc((size_t)P, sizeof(sol_t)); /* per-rank stale `path` */
    const int lastpower = 1 << (int)log2((double)P);
    char line[160];
    for (int i = 0; i < P - lastpower; i++)
    {
        snprintf(line, sizeof line, "process %i is about to receive %i cities from process %i\n", i,
                 rank[i + lastpower].len, i + lastpower);
        log_append(log, logcap, &used, line);
        if (rc == 0 && tree_receive(&acc[i], &rank[i], &rank[i + lastpower]) < 0)
            rc = -1;
    }
    for (int dd = 0; dd < (int)log2((double)lastpower); dd++)
        for (int k = 0; k < lastpower; k += 1 << (dd + 1))
            if (rc == 0 && tree_receive(&acc[k], &rank[k], &rank[k + (1 << dd)]) < 0)
                rc = -1;
    *final_cost = rank[0].cost;

    for (int r = 0; r < P; r++)
    {
        free(rank[r].p);
        free(acc[r].p);
    }
    for (int b = 0; b < B; b++)
        free(blocks[b].p);
    free(rank);
    free(acc);
    free(blocks);
    free(cnt);
    return rc;
}

/* cascade_stats.c — CPU analysis aid (not product code): classifies every
 * cascade iteration of random-action rollouts on the oracle, to size which
 * kinds of step the GPU's bitboard path could take.
 *   cc -O2 -fopenmp -o /tmp/cascade_stats tools/cascade_stats.c && /tmp/cascade_stats R C k smask envs steps
 */
#include "../oracle/tmg_oracle.c"
#include <stdio.h>

static long cnt[16], why[8];
enum { K_SIMPLE, K_LASER, K_BOMB, K_COOKIE, K_ACT, K_ACT_LASERONLY, K_COMBO, K_ITERS, K_STEPS, K_EFF, K_PERP, K_SHARED };

static int move_stats(board_t *b, int r1, int c1, int r2, int c2, long *loc) {
    if (!is_move_effective(b, r1, c1, r2, c2)) return 0;
    loc[K_EFF]++;
    const int C = b->C;
    int p = r1 * C + c1, q = r2 * C + c2;
    swap_cells(b, p, q);
    int tp = b->typ[p], tq = b->typ[q];
    if (((tp != 0 && tp != 1) && (tq != 0 && tq != 1)) || tp < 0 || tq < 0) {
        loc[K_COMBO]++;
        combination_match(b, r1, c1, r2, c2);
        gravity(b); refill(b);
    }
    lines_t L; lines_init(&L);
    matches_t M; matches_init(&M);
    for (;;) {
        if (b->err) break;
        get_colour_lines(b, &L);
        if (L.n == 0) break;
        /* shared cells between lines */
        int shared = 0;
        for (int i = 0; i < L.n && !shared; i++)
            for (int j = i + 1; j < L.n && !shared; j++)
                for (int x = 0; x < L.v[i].n && !shared; x++)
                    if (line_has(&L.v[j], L.v[i].c[x])) shared = 1;
        process_colour_lines(b, &L, &M);
        if (M.n == 0) break;
        int nact0 = b->n_act, laser = 0, bomb = 0, cookie = 0;
        for (int i = 0; i < M.n; i++) {
            if (M.name[i] == M_VLASER || M.name[i] == M_HLASER) laser = 1;
            if (M.name[i] == M_BOMB) bomb = 1;
            if (M.name[i] == M_COOKIE) cookie = 1;
        }
        /* specials sitting on matched cells */
        int sp = 0, sp_nonlaser = 0;
        for (int i = 0; i < M.n; i++)
            for (int x = 0; x < M.coords[i].n; x++) {
                int t = b->typ[M.coords[i].c[x]];
                if (t != 0 && t != 1) { sp = 1; if (t != T_VLASER && t != T_HLASER) sp_nonlaser = 1; }
            }
        /* would the GPU's wave-parallel step take it? (sb_simple_step / simple_step_lds) */
        {
            int rs = -1, perp = 0, has4 = 0, has5 = 0, ncookie = 0;
            for (int i = 0; i < L.n; i++) { int bot = L.v[i].c[L.v[i].n - 1] / b->C; if (bot > rs) rs = bot; }
            for (int i = 0; i < L.n; i++) {
                const line_t *l = &L.v[i];
                int horiz = l->n >= 2 && l->c[0] / b->C == l->c[1] / b->C;
                int bot = l->c[l->n - 1] / b->C;
                if (bot != rs) perp = 1;
                if (l->n == 4) has4 = 1;
                if (l->n >= 5) has5 = 1;
                (void)horiz;
            }
            for (int p = 0; p < b->R * b->C; p++) ncookie += b->typ[p] < 0;
            int slow = perp || cookie || (has5 && (b->smask & 1));
            int lasers = 0;
            for (int i = 0; i < M.n; i++) if (M.name[i] == M_VLASER || M.name[i] == M_HLASER) lasers = 1;
            if (shared && lasers) slow = 1;
            if (shared && (b->smask & 8)) {
                if (has4) slow = 1;
                for (int i = 0; i < L.n; i++) if (L.v[i].n > 5 && L.v[i].c[0] / b->C == L.v[i].c[1] / b->C) slow = 1;
            }
            if (sp && (ncookie || b->R * b->C > 128)) slow = 1;
            if (slow) loc[K_PERP]++;
            if (slow) {
#pragma omp atomic
                why[perp ? 0 : cookie ? 1 : (shared && lasers) ? 2 : (shared && has4) ? 3 : sp ? 4 : 5]++;
            }
        }
        resolve_colour_matches(b, &M);
        loc[K_ITERS]++;
        if (shared) loc[K_SHARED]++;
        if (sp) { loc[K_ACT]++; if (!sp_nonlaser) loc[K_ACT_LASERONLY]++; }
        else if (cookie) loc[K_COOKIE]++;
        else if (bomb) loc[K_BOMB]++;
        else if (laser) loc[K_LASER]++;
        else loc[K_SIMPLE]++;
        (void)nact0;
        gravity(b); refill(b);
    }
    lines_free(&L); matches_free(&M);
    L.n = 0;
    lines_init(&L);
    while (!b->err && (!possible_move(b) || L.n > 0)) {
        if (L.n > 0) remove_colour_lines(b, &L);
        else shuffle(b);
        get_colour_lines(b, &L);
    }
    lines_free(&L);
    {
        int ck = 0;
        for (int p = 0; p < b->R * b->C; p++) ck |= b->typ[p] < 0;
        if (ck) {
#pragma omp atomic
            why[6]++;
        }
    }
    return 0;
}

int main(int argc, char **argv) {
    int R = atoi(argv[1]), C = atoi(argv[2]), k = atoi(argv[3]), smask = atoi(argv[4]);
    long envs = atol(argv[5]); int steps = atoi(argv[6]);
    const int A = num_actions(R, C);
#pragma omp parallel
    {
        long loc[16] = {0};
        int8_t brd[2 * 512];
#pragma omp for schedule(dynamic, 8)
        for (long e = 0; e < envs; e++) {
            board_t b; bind(&b, R, C, k, smask, brd);
            uint64_t w[5] = {0x9E3779B97F4A7C15ULL * (e + 1), (uint64_t)e, 0xda3e39cb94b95bdbULL | 1, 0x5851f42d4c957f2dULL, 0};
            rng_load(&b.rng, w);
            uint64_t x = 88172645463325252ULL ^ (uint64_t)e;
            generate_board(&b);
            for (int s = 0; s < steps; s++) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                int a = (int)(x % (uint64_t)A), r1, c1, r2, c2;
                action_coords(R, C, a, &r1, &c1, &r2, &c2);
                loc[K_STEPS]++;
                move_stats(&b, r1, c1, r2, c2, loc);
                if ((s + 1) % 30 == 0) generate_board(&b);
            }
        }
#pragma omp critical
        for (int i = 0; i < 16; i++) cnt[i] += loc[i];
    }
    const char *nm[] = {"simple", "laser", "bomb", "cookie", "activation", "act_laser_only", "combo", "iters", "steps", "effective", "serial(est)", "shared"};
    for (int i = 0; i < 12; i++) printf("%-15s %10ld  %.4f per iter\n", nm[i], cnt[i], cnt[K_ITERS] ? (double)cnt[i] / cnt[K_ITERS] : 0.0);
    printf("serial reasons: perp %ld cookie %ld shared+laser %ld shared+4line(bomb) %ld act+cookie %ld other %ld; effective moves ending with a cookie on the board %ld\n", why[0], why[1], why[2], why[3], why[4], why[5], why[6]);
    return 0;
}

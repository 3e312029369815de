/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, called by, or shipped with the product
 * (libpongmi). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the reference's environment path, written from the reference's
 * semantics (not from the HIP kernels):
 *   - collide_sphere_with_moving_plane   envs/physics.py:3-23
 *   - PongEnv2P.reset                    envs/my_pong_env_2p.py:83-114
 *   - PongEnv2P.step                     envs/my_pong_env_2p.py:116-225
 *   - PongEnv2P._maybe_scale_speed       envs/my_pong_env_2p.py:227-232
 *   - PongEnv2P._get_obs_for_A/_B        envs/my_pong_env_2p.py:235-257
 *   - CPython's `random` module (MT19937 init_by_array + genrand_res53, random.uniform,
 *     randrange via getrandbits) — the global stream the reference draws its serves from.
 *
 * Pinned against the tests/golden npz fixtures, which tests/golden/make_golden.py produced by running the
 * reference itself (python -B, gym/pygame stubbed) in the build container.
 *
 * All arithmetic is IEEE binary64 in exactly the reference's evaluation order (Python evaluates
 * `a*b*c` as `(a*b)*c`); build with -ffp-contract=off so no FMA is formed.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <unistd.h>
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------ CPython MT19937 */

typedef struct {
    uint32_t mt[624];
    int mti;
} or_mt;

static void mt_init_genrand(or_mt* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = 624;
}

/* CPython Modules/_randommodule.c init_by_array */
static void mt_init_by_array(or_mt* s, const uint32_t* key, int keylen) {
    mt_init_genrand(s, 19650218u);
    int i = 1, j = 0;
    int k = 624 > keylen ? 624 : keylen;
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
        if (j >= keylen) j = 0;
    }
    for (k = 623; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
}

/* random.seed(n) for a non-negative Python int n < 2**64 */
void or_mt_seed(or_mt* s, uint64_t n) {
    uint32_t key[2];
    int keylen;
    key[0] = (uint32_t)(n & 0xffffffffu);
    key[1] = (uint32_t)(n >> 32);
    keylen = key[1] ? 2 : 1;
    mt_init_by_array(s, key, keylen);
}

uint32_t or_mt_u32(or_mt* s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    uint32_t y;
    if (s->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (s->mt[623] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
        s->mt[623] = s->mt[396] ^ (y >> 1) ^ mag01[y & 1u];
        s->mti = 0;
    }
    y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* random.random() == genrand_res53 */
double or_mt_random(or_mt* s) {
    uint32_t a = or_mt_u32(s) >> 5, b = or_mt_u32(s) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* random.uniform(a, b) (Lib/random.py: a + (b-a) * self.random()) */
double or_mt_uniform(or_mt* s, double a, double b) { return a + (b - a) * or_mt_random(s); }

/* random.randint(0, n-1) == randrange(n) == _randbelow_with_getrandbits(n), n >= 1 */
int32_t or_mt_randbelow(or_mt* s, int32_t n) {
    int k = 0;
    while ((1u << k) <= (uint32_t)n) k++; /* n.bit_length() */
    uint32_t r;
    do { r = or_mt_u32(s) >> (32 - k); } while (r >= (uint32_t)n);
    return (int32_t)r;
}

int32_t or_mt_sizeof(void) { return (int32_t)sizeof(or_mt); }

/* ------------------------------------------------------------------ physics (physics.py:3-23) */

void or_collide(double vn, double vt, double u, double omega, double e, double mu, double m, double R,
                double* out3) {
    double vn_post = (-e) * vn;                          /* - e * vn          */
    double Jn = (m * (1.0 + e)) * fabs(vn);              /* m * (1 + e) * |vn| */
    double I = ((2.0 / 5.0) * m) * pow(R, 2.0);          /* (2/5) * m * R**2   */
    double Jt_star = ((2.0 * m) / 7.0) * ((u + R * omega) - vt);
    double max_fric = mu * Jn;
    double Jt;
    if (fabs(Jt_star) <= max_fric) {
        Jt = Jt_star;
    } else {
        double vrel = (vt - u) - R * omega;
        double sgn = copysign(1.0, vrel);
        Jt = (-max_fric) * sgn;                          /* - mfi * sign       */
    }
    out3[0] = vn_post;
    out3[1] = vt + (Jt / m);
    out3[2] = omega - (R * Jt) / I;
}

/* ------------------------------------------------------------------ env (my_pong_env_2p.py) */

typedef struct {
    double paddle_width, paddle_speed, magnus_factor, restitution, friction, ball_mass, radius;
    double speed_lo, speed_hi, spin_lo, spin_hi;
    double ang0_lo, ang0_hi, ang1_lo, ang1_hi;
    double speed_increment;
    int32_t max_score, speed_scale_every, enable_spin, _pad;
} or_params;

typedef struct {
    double x, y, vx, vy, spin, top, bot;
    int32_t scoreA, scoreB, bounces, _pad;
} or_arena;

int32_t or_params_sizeof(void) { return (int32_t)sizeof(or_params); }
int32_t or_arena_sizeof(void) { return (int32_t)sizeof(or_arena); }

/* reset() serve draws, in the reference's draw order (:94-110): speed, coin, angle, spin. */
void or_reset_draws(or_mt* s, const or_params* p, double* out3 /* vx, vy, spin */) {
    double speed = or_mt_uniform(s, p->speed_lo, p->speed_hi);
    double angle_deg;
    if (or_mt_random(s) < 0.5) angle_deg = or_mt_uniform(s, p->ang0_lo, p->ang0_hi);
    else angle_deg = or_mt_uniform(s, p->ang1_lo, p->ang1_hi);
    double angle_rad = angle_deg * (3.141592653589793 / 180.0); /* math.radians */
    out3[0] = speed * cos(angle_rad);
    out3[1] = speed * sin(angle_rad);
    out3[2] = or_mt_uniform(s, p->spin_lo, p->spin_hi);
}

void or_reset_apply(or_arena* a, double vx, double vy, double spin) {
    a->scoreA = 0; a->scoreB = 0; a->bounces = 0;
    a->top = 0.5; a->bot = 0.5;
    a->x = 0.5; a->y = 0.5;
    a->vx = vx; a->vy = vy; a->spin = spin;
}

void or_obs(const or_arena* a, float* obsA, float* obsB) {
    obsA[0] = (float)a->x; obsA[1] = (float)(1.0 - a->y); obsA[2] = (float)a->vx; obsA[3] = (float)(-a->vy);
    obsA[4] = (float)a->top; obsA[5] = (float)a->bot; obsA[6] = (float)a->spin;
    obsB[0] = (float)a->x; obsB[1] = (float)a->y; obsB[2] = (float)a->vx; obsB[3] = (float)a->vy;
    obsB[4] = (float)a->bot; obsB[5] = (float)a->top; obsB[6] = (float)a->spin;
}

static double clip01(double v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); } /* np.clip(v,0,1) */

static void maybe_scale(const or_params* p, or_arena* a) {
    if (a->bounces % p->speed_scale_every == 0) {
        double scale = 1.0 + p->speed_increment;
        a->vx = a->vx * scale;
        a->vy = a->vy * scale;
    }
}

/* One tick. Returns done. rewards[0]=rA, rewards[1]=rB. */
int32_t or_step(const or_params* p, or_arena* a, int32_t aA, int32_t aB, float* rew2) {
    if (aA == 0) a->top = a->top - p->paddle_speed;
    else if (aA == 2) a->top = a->top + p->paddle_speed;
    a->top = clip01(a->top);
    if (aB == 0) a->bot = a->bot - p->paddle_speed;
    else if (aB == 2) a->bot = a->bot + p->paddle_speed;
    a->bot = clip01(a->bot);

    double rA = 0.0, rB = 0.0;
    int32_t done = 0;

    if (p->enable_spin) a->vx = a->vx + (p->magnus_factor * a->spin) * a->vy;
    a->x = a->x + a->vx;
    a->y = a->y + a->vy;

    if (a->x < 0.0) { a->x = -a->x; a->vx = -a->vx; }
    else if (a->x > 1.0) { a->x = 2.0 - a->x; a->vx = -a->vx; }

    double half = p->paddle_width / 2.0;
    double out[3];
    if (a->y < 0.0) {
        double lo = a->top - half, hi = a->top + half;
        if (lo <= a->x && a->x <= hi) {
            double u = 0.0;
            if (aA == 0) u = -p->paddle_speed; else if (aA == 2) u = p->paddle_speed;
            or_collide(a->vy, a->vx, u, a->spin, p->restitution, p->friction, p->ball_mass, p->radius, out);
            a->vy = out[0]; a->vx = out[1]; a->spin = out[2];
            a->y = 0.0;
            a->bounces += 1;
            maybe_scale(p, a);
        } else {
            rA -= 1.0; rB += 1.0;
            a->scoreB += 1;
            if (a->scoreB >= p->max_score) done = 1;
        }
    } else if (a->y > 1.0) {
        double lo = a->bot - half, hi = a->bot + half;
        if (lo <= a->x && a->x <= hi) {
            double u = 0.0;
            if (aB == 0) u = -p->paddle_speed; else if (aB == 2) u = p->paddle_speed;
            or_collide(-a->vy, a->vx, u, a->spin, p->restitution, p->friction, p->ball_mass, p->radius, out);
            a->vy = -out[0]; a->vx = out[1]; a->spin = out[2];
            a->y = 1.0;
            a->bounces += 1;
            maybe_scale(p, a);
        } else {
            rA += 1.0; rB -= 1.0;
            a->scoreA += 1;
            if (a->scoreA >= p->max_score) done = 1;
        }
    }
    rew2[0] = (float)rA;
    rew2[1] = (float)rB;
    return done;
}

/* ------------------------------------------------------------------ batched helpers for tests */

/* Advance n independent arenas one tick with given actions (no reset). Arrays are SoA-ish:
 * arenas[n], aA/aB[n], obsA/obsB[n*7], rew[n*2], done[n]. */
void or_step_batch(const or_params* p, or_arena* arenas, const int8_t* aA, const int8_t* aB,
                   float* obsA, float* obsB, float* rew, uint8_t* done, int32_t n) {
    for (int32_t i = 0; i < n; i++) {
        done[i] = (uint8_t)or_step(p, &arenas[i], aA[i], aB[i], rew + 2 * i);
        or_obs(&arenas[i], obsA + 7 * i, obsB + 7 * i);
    }
}

/* Config-1 CPU loop (BASELINE.json configs[0]): one arena, random-vs-random with the CPython
 * stream (`random.seed(seed)`, actions by randint(0,2) for A then B, reset on done, serves from
 * the same stream — exactly the reference loop of tests/arena.py:294-320 with random agents).
 * Returns the number of completed episodes; steps are always `steps`. */
int64_t or_rollout_random(const or_params* p, uint64_t seed, int64_t steps, int64_t* score_sum) {
    or_mt s;
    or_arena a;
    double d[3];
    float rew[2];
    int64_t episodes = 0, ssum = 0;
    or_mt_seed(&s, seed);
    or_reset_draws(&s, p, d);
    or_reset_apply(&a, d[0], d[1], d[2]);
    for (int64_t t = 0; t < steps; t++) {
        int32_t aA = or_mt_randbelow(&s, 3);
        int32_t aB = or_mt_randbelow(&s, 3);
        if (or_step(p, &a, aA, aB, rew)) {
            episodes++;
            ssum += a.scoreA - a.scoreB;
            or_reset_draws(&s, p, d);
            or_reset_apply(&a, d[0], d[1], d[2]);
        }
    }
    if (score_sum) *score_sum = ssum;
    return episodes;
}

/* ------------------------------------------------------------------ QNet forward, float32 tile order */
/*
 * QNet.forward (models/qnet.py:71-75: ReLU(W1 x + b1) -> ReLU(W2 h + b2) -> V, A heads,
 * Q = V + (A - A.mean(1))) evaluated in IEEE binary32 in ONE fixed order: the order libpongmi's
 * matrix-core tile uses, where v_mfma_f32_32x32x2_f32 is bitwise a k-ordered fmaf chain
 * (MI355X_MICROARCH.md, F32 MFMA row). torch itself fixes no summation order for these products
 * (BLAS-dependent), so any order is a valid float32 evaluation of the reference; restating the
 * device's one lets the tests compare every argmax (every action of every arena) exactly instead of
 * skipping near-ties. The tie to the reference's own outputs is the Q tolerance test against the
 * golden fixture (tests/golden/qnet.npz, made by running models/qnet.py).
 *
 * Order per output (w = the effective-weight block of include/pongmi.h, plain part):
 *   layer 1, unit j:  acc = fmaf(b1[j], 1, +0); acc = fmaf(W1[j][k], x[k], acc) for k = 0..6
 *   layer 2, unit j:  acc = b2[j]; for t in {0,1}, r in 0..15, u = 32t + (r&3) + 8(r>>2):
 *                       acc = fmaf(W2[j][u], h1[u], acc); acc = fmaf(W2[j][u+4], h1[u+4], acc)
 *   head c (V, A0..A2): two half sums s_h (h = 0, 1) over u = 32t + (r&3) + 8(r>>2) + 4h in the same
 *                       (t, r) order, s_h = fmaf(Wh[c][u], relu(h2[u]), s_h) from +0; then
 *                       (s_0 + s_1) + bh[c]
 *   mean = ((A0 + A1) + A2) / 3;  Q_c = V + (A_c - mean)
 * ReLU maps every negative float (sign bit set, -0 included) to +0.
 * Outputs: q [n][3]; feat (nullable) [n][64] the pre-ReLU layer-2 values.
 */
#define OR_QW1 0
#define OR_QB1 448
#define OR_QW2 512
#define OR_QB2 4608
#define OR_QWH 4672
#define OR_QBH 4928

static float relu_f32(float x) {
    int32_t i;
    memcpy(&i, &x, 4);
    if (i < 0) i = 0;
    memcpy(&x, &i, 4);
    return x;
}

static void qnet_rows(const float* w, const float* obs, int32_t i0, int32_t i1, float* q, float* feat) {
    for (int32_t i = i0; i < i1; i++) {
        const float* x = obs + 7 * (int64_t)i;
        float h1[64], h2[64], hs[4];
        for (int j = 0; j < 64; j++) {
            float acc = fmaf(w[OR_QB1 + j], 1.0f, 0.0f);
            for (int k = 0; k < 7; k++) acc = fmaf(w[OR_QW1 + 7 * j + k], x[k], acc);
            h1[j] = relu_f32(acc);
        }
        for (int j = 0; j < 64; j++) {
            const float* row = w + OR_QW2 + 64 * j;
            float acc = w[OR_QB2 + j];
            for (int t = 0; t < 2; t++)
                for (int r = 0; r < 16; r++) {
                    const int u = 32 * t + (r & 3) + 8 * (r >> 2);
                    acc = fmaf(row[u], h1[u], acc);
                    acc = fmaf(row[u + 4], h1[u + 4], acc);
                }
            h2[j] = acc;
            if (feat) feat[64 * (int64_t)i + j] = acc;
        }
        for (int c = 0; c < 4; c++) {
            float s[2];
            for (int h = 0; h < 2; h++) {
                float acc = 0.0f;
                for (int t = 0; t < 2; t++)
                    for (int r = 0; r < 16; r++) {
                        const int u = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
                        acc = fmaf(w[OR_QWH + 64 * c + u], relu_f32(h2[u]), acc);
                    }
                s[h] = acc;
            }
            hs[c] = (s[0] + s[1]) + w[OR_QBH + c];
        }
        const float mean = ((hs[1] + hs[2]) + hs[3]) / 3.0f;
        for (int c = 0; c < 3; c++) q[3 * (int64_t)i + c] = hs[0] + (hs[1 + c] - mean);
    }
}

typedef struct {
    const float *w, *obs;
    int32_t i0, i1;
    float *q, *feat;
} qnet_job;

static void* qnet_job_run(void* p) {
    const qnet_job* j = (const qnet_job*)p;
    qnet_rows(j->w, j->obs, j->i0, j->i1, j->q, j->feat);
    return NULL;
}

/* Rows are independent: large batches are split over up to 16 threads (each row's arithmetic, and so
 * every output bit, is the same whichever thread computes it). */
void or_qnet_f32(const float* w, const float* obs, int32_t n, float* q, float* feat) {
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    if (nt > 16) nt = 16;
    if (n < 4096 || nt < 2) {
        qnet_rows(w, obs, 0, n, q, feat);
        return;
    }
    pthread_t th[16];
    qnet_job jobs[16];
    const int32_t per = (int32_t)((n + nt - 1) / nt);
    int started = 0;
    for (long t = 0; t < nt; t++) {
        const int32_t i0 = (int32_t)(t * per), i1 = i0 + per < n ? i0 + per : n;
        jobs[t] = (qnet_job){w, obs, i0, i1 > i0 ? i1 : i0, q, feat};
        if (t > 0 && pthread_create(&th[t], NULL, qnet_job_run, &jobs[t]) == 0) started |= 1 << t;
        else if (t > 0) qnet_job_run(&jobs[t]);
    }
    qnet_job_run(&jobs[0]);
    for (long t = 1; t < nt; t++)
        if (started & (1 << t)) pthread_join(th[t], NULL);
}

/* torch argmax over [n][3] (first maximal index), as an int8 action row. */
void or_argmax3(const float* q, int32_t n, int8_t* a) {
    for (int32_t i = 0; i < n; i++) {
        const float* r = q + 3 * (int64_t)i;
        int b = 0;
        if (r[1] > r[b]) b = 1;
        if (r[2] > r[b]) b = 2;
        a[i] = (int8_t)b;
    }
}

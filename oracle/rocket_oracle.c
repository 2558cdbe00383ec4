/*
 * rocket_oracle.c — TEST INFRASTRUCTURE ONLY. See rocket_oracle.h for scope and
 * for who may load it. Every function cites the reference (or the pinned
 * third-party algorithm) it restates. fp64 throughout, except where the
 * reference itself computes in float32 (noted inline).
 */
#include "rocket_oracle.h"

#include <float.h>
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NMAX 14
#define EPS DBL_EPSILON

/* ---------------------------------------------------------------------------
 * Physical constants of the reference simulators.
 *   6DOF: simulator.py:210-224 (g0, J, Isp, r_T_B = [-15,0,0]; aero force is 0, :359-360)
 *   3DOF: simulator.py:36-51  (g0, I, Isp, Cd = 0.3, Sref, x_CG, x_CP, x_T; alpha = 0)
 * ------------------------------------------------------------------------- */
static const double G0 = 9.81;
static const double ISP = 360.0;
static const double J6[3] = {75350.25, 6037675.13, 6037675.13};
static const double RT6 = -15.0;
static const double I3 = 6.04e6, SREF3 = 10.5, CD3 = 0.3, RHO3 = 1.225;
static const double XCG3 = 10.0, XCP3 = 20.0, XT3 = 40.0;

/* ---------------------------------------------------------------------------
 * Controls, fixed for one env step.
 * ------------------------------------------------------------------------- */
typedef struct ctrl {
    int model;
    /* 6DOF: thrust in body frame, simulator.py:311-318 + :350-357.
     * np.cos/np.sin of a float32 gimbal return float32 and the products
     * cos*cos, sin*cos are float32 products; the matrix-vector product with
     * [T, 0, 0] is then fp64 (ROT_MAT is built as a float64 array). */
    double tb[3];
    double dm;         /* -T/(g0*Isp), simulator.py:291-292 */
    /* 3DOF: simulator.py:94-130 */
    double delta;      /* float32 gimbal promoted */
    double thrust;
    double dom3;       /* (N*(xcg-xcp) - T*sin(delta)*(xT-xCG))/I with N = 0 */
} ctrl;

static void make_ctrl(const ro_cfg* c, const float* u, ctrl* k)
{
    k->model = c->model;
    if (c->model == 6) {
        float dy = u[0], dz = u[1], T = u[2];
        float cy = cosf(dy), sy = sinf(dy), cz = cosf(dz), sz = sinf(dz);
        float p0 = cy * cz, p1 = sy * cz;           /* float32 products */
        k->tb[0] = (double)p0 * (double)T;
        k->tb[1] = (double)p1 * (double)T;
        k->tb[2] = (double)sz * (double)T;
        k->dm = -(double)T / (G0 * ISP);
    } else {
        float d = u[0], T = u[1];
        float sd = sinf(d);
        float tsd = T * sd;                          /* float32: T*np.sin(delta) */
        k->delta = (double)d;
        k->thrust = (double)T;
        /* legacy (numpy 1.x) promotion of float32 * python int -> float64 */
        k->dom3 = (0.0 * (XCG3 - XCP3) - (double)tsd * (XT3 - XCG3)) / I3;
        k->dm = -(double)T / (ISP * G0);
    }
}

/* 6DOF RHS, simulator.py:259-294. */
static void rhs6(const ctrl* k, const double* y, double* dy)
{
    const double q0 = y[6], q1 = y[7], q2 = y[8], q3 = y[9];
    /* Rotation.from_quat([q1,q2,q3,q0]) normalises, then as_matrix (simulator.py:337-347) */
    double nrm = sqrt(q1 * q1 + q2 * q2 + q3 * q3 + q0 * q0);
    double x = q1 / nrm, yy = q2 / nrm, z = q3 / nrm, w = q0 / nrm;
    double x2 = x * x, y2 = yy * yy, z2 = z * z, w2 = w * w;
    double xy = x * yy, zw = z * w, xz = x * z, yw = yy * w, yz = yy * z, xw = x * w;
    double R[3][3];
    R[0][0] = x2 - y2 - z2 + w2;
    R[1][0] = 2 * (xy + zw);
    R[2][0] = 2 * (xz - yw);
    R[0][1] = 2 * (xy - zw);
    R[1][1] = -x2 + y2 - z2 + w2;
    R[2][1] = 2 * (yz + xw);
    R[0][2] = 2 * (xz + yw);
    R[1][2] = 2 * (yz - xw);
    R[2][2] = -x2 - y2 + z2 + w2;
    const double* tb = k->tb;
    double inv_m = 1.0 / y[13];                     /* 1/mass*F_I + g_I, :281 */
    for (int i = 0; i < 3; ++i) {
        double F = R[i][0] * tb[0] + R[i][1] * tb[1] + R[i][2] * tb[2];
        dy[i] = y[3 + i];
        dy[3 + i] = inv_m * F + (i == 0 ? -G0 : 0.0);
    }
    /* dq = 0.5*OMEGA(omega).q with the UNnormalised q, :284-287, :362-370 */
    const double w1 = y[10], w2_ = y[11], w3 = y[12];
    dy[6] = 0.5 * (-w1 * q1 - w2_ * q2 - w3 * q3);
    dy[7] = 0.5 * (w1 * q0 + w3 * q2 - w2_ * q3);
    dy[8] = 0.5 * (w2_ * q0 - w3 * q1 + w1 * q3);
    dy[9] = 0.5 * (w3 * q0 + w2_ * q1 - w1 * q2);
    /* torques = r_T_B x T_b (aero term is zero), :373-378; r_T_B = [-15,0,0] */
    double tau[3] = {0.0 * tb[2] - 0.0 * tb[1], 0.0 * tb[0] - RT6 * tb[2], RT6 * tb[1] - 0.0 * tb[0]};
    double Jw[3] = {J6[0] * w1, J6[1] * w2_, J6[2] * w3};
    double cr[3] = {w2_ * Jw[2] - w3 * Jw[1], w3 * Jw[0] - w1 * Jw[2], w1 * Jw[1] - w2_ * Jw[0]};
    for (int i = 0; i < 3; ++i) dy[10 + i] = (1.0 / J6[i]) * (tau[i] - cr[i]);
    dy[13] = k->dm;
}

/* 3DOF RHS, simulator.py:88-130 (alpha = 0 => N = 0; Cd = 0.3; the z-drag uses
 * cos(phi): reference quirk, reproduced). */
static void rhs3(const ctrl* k, const double* y, double* dy)
{
    const double phi = y[2], vx = y[3], vz = y[4];
    double v2 = vx * vx + vz * vz;
    double Q = 0.5 * RHO3 * v2;
    double A = CD3 * Q * SREF3;
    double N = 0.0 * Q * SREF3;
    double T = k->thrust;
    double ax = (T * cos(k->delta + phi) - N * sin(phi) - A * cos(phi)) / y[6];
    double az = (T * sin(k->delta + phi) + N * cos(phi) - A * cos(phi)) / y[6] - G0;
    dy[0] = vx;
    dy[1] = vz;
    dy[2] = y[5];
    dy[3] = ax;
    dy[4] = az;
    dy[5] = k->dom3;
    dy[6] = k->dm;
}

static void rhs(const ctrl* k, const double* y, double* dy)
{
    if (k->model == 6) rhs6(k, y, dy);
    else rhs3(k, y, dy);
}

void ro_rhs(const ro_cfg* c, const double* y, const float* u, double* dy)
{
    ctrl k;
    make_ctrl(c, u, &k);
    rhs(&k, y, dy);
}

/* ---------------------------------------------------------------------------
 * scipy RK45 (Dormand–Prince), restated from scipy.integrate._ivp.rk (identical
 * text in 1.7.1 and 1.15.3): tableau RK45.C/A/B/E/P, rk_step, _step_impl.
 * ------------------------------------------------------------------------- */
/* (RK45.C is not needed: both RHS are autonomous, simulator.py:259, :88) */
static const double DA[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
static const double DB[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
static const double DE[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525,
                             1.0 / 40};
static const double DP[7][4] = {
    {1, -8048581381.0 / 2820520608, 8663915743.0 / 2820520608, -12715105075.0 / 11282082432},
    {0, 0, 0, 0},
    {0, 131558114200.0 / 32700410799, -68118460800.0 / 10900136933, 87487479700.0 / 32700410799},
    {0, -1754552775.0 / 470086768, 14199869525.0 / 1410260304, -10690763975.0 / 1880347072},
    {0, 127303824393.0 / 49829197408, -318862633887.0 / 49829197408, 701980252875.0 / 199316789632},
    {0, -282668133.0 / 205662961, 2019193451.0 / 616988883, -1453857185.0 / 822651844},
    {0, 40617522.0 / 29380423, -110615467.0 / 29380423, 69997945.0 / 29380423}};

static const double SAFETY = 0.9, MIN_FACTOR = 0.2, MAX_FACTOR = 10.0;
static const double RTOL = 1e-3, ATOL = 1e-6;

/* common.norm: np.linalg.norm(x) / sqrt(n) */
static double rms(const double* x, int n)
{
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[i] * x[i];
    return sqrt(s) / sqrt((double)n);
}

typedef struct solver {
    const ctrl* k;
    int n;
    double t, t_bound, t_old, h_abs;
    double y[NMAX], f[NMAX], y_old[NMAX];
    double K[7][NMAX];
    int nfev;
} solver;

static void feval(solver* s, const double* y, double* dy)
{
    rhs(s->k, y, dy);
    s->nfev++;
}

/* common.select_initial_step (scipy 1.7: return min(100*h0, h1); scipy >= 1.12 also
 * clamps h0 and the result to the interval length). */
static double select_initial_step(solver* s, int clamp)
{
    const int n = s->n;
    double sc[NMAX], tmp[NMAX], y1[NMAX], f1[NMAX];
    double interval = fabs(s->t_bound - s->t);
    if (clamp && interval == 0.0) return 0.0;
    for (int i = 0; i < n; ++i) sc[i] = ATOL + fabs(s->y[i]) * RTOL;
    for (int i = 0; i < n; ++i) tmp[i] = s->y[i] / sc[i];
    double d0 = rms(tmp, n);
    for (int i = 0; i < n; ++i) tmp[i] = s->f[i] / sc[i];
    double d1 = rms(tmp, n);
    double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    if (clamp && h0 > interval) h0 = interval;
    for (int i = 0; i < n; ++i) y1[i] = s->y[i] + h0 * 1.0 * s->f[i];
    feval(s, y1, f1);
    for (int i = 0; i < n; ++i) tmp[i] = (f1[i] - s->f[i]) / sc[i];
    double d2 = rms(tmp, n) / h0;
    double h1;
    if (d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
    else h1 = pow(0.01 / fmax(d1, d2), 1.0 / (4 + 1));
    double r = fmin(100 * h0, h1);
    if (clamp) r = fmin(r, interval); /* max_step = inf */
    return r;
}

/* rk.rk_step */
static void rk_step(solver* s, double h, double* y_new, double* f_new)
{
    const int n = s->n;
    double yt[NMAX];
    memcpy(s->K[0], s->f, sizeof(double) * n);
    for (int st = 1; st < 6; ++st) {
        for (int i = 0; i < n; ++i) {
            double dy = 0.0;
            for (int j = 0; j < st; ++j) dy += s->K[j][i] * DA[st][j];
            yt[i] = s->y[i] + dy * h;
        }
        feval(s, yt, s->K[st]);
    }
    for (int i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int j = 0; j < 6; ++j) acc += s->K[j][i] * DB[j];
        y_new[i] = s->y[i] + h * acc;
    }
    feval(s, y_new, f_new);
    memcpy(s->K[6], f_new, sizeof(double) * n);
}

/* rk.RungeKutta._step_impl; returns 0 on TOO_SMALL_STEP failure. */
static int step_impl(solver* s)
{
    const int n = s->n;
    double t = s->t;
    double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
    double h_abs = s->h_abs < min_step ? min_step : s->h_abs; /* max_step = inf */
    int rejected = 0;
    double y_new[NMAX], f_new[NMAX], err[NMAX];
    for (;;) {
        /* scipy: `if h_abs < min_step: return False, TOO_SMALL_STEP`. A NaN h_abs (non-finite
         * state or action) fails that test for ever and scipy's step never returns; written
         * negated, the restatement ends it as TOO_SMALL_STEP (status -1 => done), as the
         * kernels do (rocket_dopri5.inc solve(), rocket_hip.hip nonfinite()). Finite h_abs:
         * identical. */
        if (!(h_abs >= min_step)) return 0;
        double t_new = t + h_abs;
        if (t_new - s->t_bound > 0) t_new = s->t_bound;
        double h = t_new - t;
        h_abs = fabs(h);
        rk_step(s, h, y_new, f_new);
        for (int i = 0; i < n; ++i) {
            double sc = ATOL + fmax(fabs(s->y[i]), fabs(y_new[i])) * RTOL;
            double e = 0.0;
            for (int j = 0; j < 7; ++j) e += s->K[j][i] * DE[j];
            err[i] = e * h / sc;
        }
        double en = rms(err, n);
        if (en < 1) {
            double factor = (en == 0) ? MAX_FACTOR : fmin(MAX_FACTOR, SAFETY * pow(en, -1.0 / 5));
            if (rejected) factor = fmin(1.0, factor);
            h_abs *= factor;
            memcpy(s->y_old, s->y, sizeof(double) * n);
            s->t_old = t;
            s->t = t_new;
            memcpy(s->y, y_new, sizeof(double) * n);
            memcpy(s->f, f_new, sizeof(double) * n);
            s->h_abs = h_abs;
            return 1;
        }
        h_abs *= fmax(MIN_FACTOR, SAFETY * pow(en, -1.0 / 5));
        rejected = 1;
    }
}

/* RkDenseOutput._call_impl: y_old + h * Q.p, p = cumprod([x]*4), Q = K^T P */
typedef struct dense {
    double t_old, h;
    const double* y_old;
    double Q[NMAX][4];
    int n;
} dense;

static void dense_init(dense* d, const solver* s)
{
    d->t_old = s->t_old;
    d->h = s->t - s->t_old;
    d->y_old = s->y_old;
    d->n = s->n;
    for (int i = 0; i < s->n; ++i)
        for (int c = 0; c < 4; ++c) {
            double q = 0.0;
            for (int j = 0; j < 7; ++j) q += s->K[j][i] * DP[j][c];
            d->Q[i][c] = q;
        }
}

static double dense_comp(const dense* d, double t, int i)
{
    double x = (t - d->t_old) / d->h;
    double p1 = x, p2 = p1 * x, p3 = p2 * x, p4 = p3 * x;
    return d->h * (d->Q[i][0] * p1 + d->Q[i][1] * p2 + d->Q[i][2] * p3 + d->Q[i][3] * p4) + d->y_old[i];
}

/* scipy.optimize brentq (Brent 1973, as implemented in scipy's Zeros/brentq.c),
 * xtol = rtol = 4*EPS (ivp.solve_event_equation), maxiter 100. */
static double brentq_dense(const dense* d, int idx, double xa, double xb)
{
    const double xtol = 4 * EPS, rtol = 4 * EPS;
    double xpre = xa, xcur = xb, xblk = 0.0, fblk = 0.0, spre = 0.0, scur = 0.0;
    double fpre = dense_comp(d, xpre, idx), fcur = dense_comp(d, xcur, idx);
    if (fpre == 0) return xpre;
    if (fcur == 0) return xcur;
    for (int it = 0; it < 100; ++it) {
        if (fpre != 0 && fcur != 0 && (signbit(fpre) != signbit(fcur))) {
            xblk = xpre;
            fblk = fpre;
            spre = scur = xcur - xpre;
        }
        if (fabs(fblk) < fabs(fcur)) {
            xpre = xcur; xcur = xblk; xblk = xpre;
            fpre = fcur; fcur = fblk; fblk = fpre;
        }
        double delta = (xtol + rtol * fabs(xcur)) / 2;
        double sbis = (xblk - xcur) / 2;
        if (fcur == 0 || fabs(sbis) < delta) return xcur;
        if (fabs(spre) > delta && fabs(fcur) < fabs(fpre)) {
            double stry;
            if (xpre == xblk) {
                stry = -fcur * (xcur - xpre) / (fcur - fpre);
            } else {
                double dpre = (fpre - fcur) / (xpre - xcur);
                double dblk = (fblk - fcur) / (xblk - xcur);
                stry = -fcur * (fblk * dblk - fpre * dpre) / (dblk * dpre * (fblk - fpre));
            }
            if (2 * fabs(stry) < fmin(fabs(spre), 3 * fabs(sbis) - delta)) {
                spre = scur;
                scur = stry;
            } else {
                spre = sbis;
                scur = sbis;
            }
        } else {
            spre = sbis;
            scur = sbis;
        }
        xpre = xcur;
        fpre = fcur;
        if (fabs(scur) > delta) xcur += scur;
        else xcur += (sbis > 0 ? delta : -delta);
        fcur = dense_comp(d, xcur, idx);
    }
    return xcur;
}

/* ivp.solve_ivp main loop with one terminal, direction-0 event g(y) = y[idx]
 * (simulator.py:230-241 6DOF idx 0; :58-69 3DOF idx 1). Returns the status
 * (0 finished, 1 terminal event, -1 failed) and the state y[-1] of solution.y. */
static int solve_ivp_rk45(const ro_cfg* c, const ctrl* k, int n, int idx, double t0, const double* y0,
                          double* y_out, int* nfev)
{
    solver s;
    memset(&s, 0, sizeof(s));
    s.k = k;
    s.n = n;
    s.t = t0;
    s.t_bound = t0 + c->dt;
    memcpy(s.y, y0, sizeof(double) * n);
    feval(&s, s.y, s.f);
    s.h_abs = select_initial_step(&s, c->scipy_clamp_h0);
    double g = s.y[idx];
    int status = -2; /* None */
    int finished = 0;
    memcpy(y_out, s.y, sizeof(double) * n);
    while (status == -2) {
        /* OdeSolver.step */
        if (s.t == s.t_bound) {
            s.t_old = s.t;
            finished = 1;
        } else {
            if (!step_impl(&s)) {
                status = -1;
                break;
            }
            if (s.t - s.t_bound >= 0) finished = 1;
        }
        if (finished) status = 0;
        memcpy(y_out, s.y, sizeof(double) * n);
        double g_new = s.y[idx];
        int up = (g <= 0) && (g_new >= 0);
        int down = (g >= 0) && (g_new <= 0);
        if (up || down) {
            dense d;
            dense_init(&d, &s);
            double root = brentq_dense(&d, idx, s.t_old, s.t);
            status = 1;
            double x = (root - d.t_old) / d.h;
            double p1 = x, p2 = p1 * x, p3 = p2 * x, p4 = p3 * x;
            for (int i = 0; i < n; ++i)
                y_out[i] = d.h * (d.Q[i][0] * p1 + d.Q[i][1] * p2 + d.Q[i][2] * p3 + d.Q[i][3] * p4) +
                           d.y_old[i];
        }
        g = g_new;
    }
    *nfev = s.nfev;
    return status;
}

/* Explicit Euler step (RO_INT_EULER, rocket_oracle.h): one RHS evaluation (simulator.py:259-294 /
 * :88-130), the terminal altitude event (the sign-change test of solve_ivp's find_active_events,
 * ivp.py, as used at simulator.py:230-241 / :58-69) with its root on Euler's linear continuous
 * extension, every component evaluated there. */
static int euler_step(const ro_cfg* c, const ctrl* k, int n, int idx, const double* y0, double* y_out,
                      int* nfev)
{
    double f0[NMAX];
    rhs(k, y0, f0);
    *nfev = 1;
    for (int i = 0; i < n; ++i) y_out[i] = y0[i] + c->dt * f0[i];
    const double g0 = y0[idx], g1 = y_out[idx];
    int status = 0;
    if ((g0 <= 0 && g1 >= 0) || (g0 >= 0 && g1 <= 0)) {
        status = 1;
        if (g1 != 0) { /* a root at the step end keeps y1 */
            const double s = g0 / (g0 - g1);
            for (int i = 0; i < n; ++i) y_out[i] = y0[i] + (s * c->dt) * f0[i];
        }
    }
    for (int i = 0; i < n; ++i)
        if (!isfinite(y_out[i])) status = status ? status : -1;
    return status;
}

/* ---------------------------------------------------------------------------
 * Env layer.
 * ------------------------------------------------------------------------- */

/* _denormalize_action, rocket_env.py:969-981 (6DOF) / :395-406 (3DOF): no clip,
 * result cast to float32. */
static void denorm_action(const ro_cfg* c, const float* a, float* u)
{
    if (c->model == 6) {
        u[0] = (float)((double)a[0] * c->max_gimbal);
        u[1] = (float)((double)a[1] * c->max_gimbal);
        u[2] = (float)(((double)a[2] + 1) / 2.0 * c->max_thrust);
    } else {
        u[0] = (float)((double)a[0] * c->max_gimbal);
        u[1] = (float)(((double)a[1] + 1) / 2.0 * c->max_thrust);
    }
}

/* Rotation.as_euler("zyx") of the (float32) attitude quaternion, closed form of the
 * extrinsic z-y-x sequence: a = atan2(-R01, R00), b = asin(R02), c = atan2(-R12, R22). */
static void euler_zyx(const float* q32, double* e)
{
    double w = q32[0], x = q32[1], y = q32[2], z = q32[3];
    double nrm = sqrt(x * x + y * y + z * z + w * w);
    x /= nrm; y /= nrm; z /= nrm; w /= nrm;
    double R00 = x * x - y * y - z * z + w * w;
    double R01 = 2 * (x * y - z * w);
    double R02 = 2 * (x * z + y * w);
    double R12 = 2 * (y * z - x * w);
    double R22 = -x * x - y * y + z * z + w * w;
    if (R02 > 1) R02 = 1;
    if (R02 < -1) R02 = -1;
    e[0] = atan2(-R01, R00);
    e[1] = asin(R02);
    e[2] = atan2(-R12, R22);
}

static double norm3(double a, double b, double c) { return sqrt(a * a + b * b + c * c); }

/* Rocket6DOF.step post-processing, rocket_env.py:690-719, 825-859, 986-1014, 1036-1061 */
static void env6_finish(const ro_cfg* c, const float* ic, const float* u, int status, const double* s64,
                        ro_out* o)
{
    float s[14];
    for (int i = 0; i < 14; ++i) s[i] = (float)s64[i];
    /* _check_bounds_violation: Box(lo,hi,float32).contains(float32(r)), inclusive, NaN -> outside */
    int inside = 1;
    for (int i = 0; i < 3; ++i)
        if (!(s[i] >= c->bounds_lo[i] && s[i] <= c->bounds_hi[i])) inside = 0;
    int bv = !inside;
    o->done = (status != 0) || bv;
    o->bounds_violation = bv;
    /* _compute_vtarg (v_0 = ||IC[3:6]|| of the float32 episode IC) */
    float v0 = sqrtf(ic[3] * ic[3] + ic[4] * ic[4] + ic[5] * ic[5]);
    double rx = s[0];
    double rh[3], vh[3], tau;
    if (rx > c->waypoint) {
        rh[0] = (double)s[0] - c->waypoint; rh[1] = s[1]; rh[2] = s[2];
        vh[0] = (double)s[3] + 2; vh[1] = s[4]; vh[2] = s[5];
        tau = 20;
    } else {
        rh[0] = (double)s[0] + 1; rh[1] = 0; rh[2] = 0;
        vh[0] = (double)s[3] + 1; vh[1] = s[4]; vh[2] = s[5];
        tau = 100;
    }
    double nrh = norm3(rh[0], rh[1], rh[2]);
    double t_go = nrh / norm3(vh[0], vh[1], vh[2]);
    double f = -(double)v0 / fmax(1e-3, nrh) * (1 - exp(-t_go / tau));
    double vt[3] = {f * rh[0], f * rh[1], f * rh[2]};
    double vel = c->alfa * norm3(s[3] - vt[0], s[4] - vt[1], s[5] - vt[2]);
    double thr = c->beta * (double)u[2];
    double e[3];
    euler_zyx(&s[6], e);
    int att = 0;
    for (int i = 0; i < 3; ++i)
        if (fabs(e[i]) > c->att_limit[i]) att = 1;
    double attitude = c->gamma * att;
    /* _check_landing (any() on attitude and omega: reference quirk) */
    double r = norm3(s[0], s[1], s[2]), v = norm3(s[3], s[4], s[5]);
    int att_ok = 0, om_ok = 0;
    for (int i = 0; i < 3; ++i) {
        if (fabs(e[i]) < c->land_att_limit[i]) att_ok = 1;
        if (fabsf(s[10 + i]) < c->omega_lim[i]) om_ok = 1;
    }
    int landing = (s[0] <= 1e-3) && (v < c->max_velocity) && (r < c->landing_radius) && att_ok && om_ok;
    double goal = c->kappa * landing;
    o->terms[0] = vel;
    o->terms[1] = thr;
    o->terms[2] = c->eta;
    o->terms[3] = attitude;
    o->terms[4] = goal;
    o->terms[5] = 0;
    o->reward = vel + thr + c->eta + attitude + goal + (bv ? -50.0 : 0.0);
    /* _get_obs: float32(state64 / normalizer) from the fp64 SIM state */
    for (int i = 0; i < 14; ++i) o->obs[i] = (float)(s64[i] / c->normalizer[i]);
}

/* Rocket.step post-processing (3DOF), rocket_env.py:150-247, 431-476 */
static void env3_finish(const ro_cfg* c, const float* ic, const float* u, int status, const double* s64,
                        ro_out* o)
{
    float s[7];
    for (int i = 0; i < 7; ++i) s[i] = (float)s64[i];
    int outside = 0;
    if (s[0] <= -c->x_bound || s[0] >= c->x_bound) outside = 1;
    if (s[1] >= c->z_bound) outside = 1;
    o->done = (status != 0) || outside;
    o->bounds_violation = outside;
    float v0 = sqrtf(ic[3] * ic[3] + ic[4] * ic[4]);
    double rz = s[1];
    double rh[2], vh[2], tau;
    if (rz > c->waypoint) {
        rh[0] = s[0]; rh[1] = (double)s[1] - c->waypoint;
        vh[0] = s[3]; vh[1] = (double)s[4] + 2;
        tau = 20;
    } else {
        rh[0] = 0; rh[1] = s[1];
        vh[0] = s[3]; vh[1] = (double)s[4] + 1;
        tau = 100;
    }
    double nrh = sqrt(rh[0] * rh[0] + rh[1] * rh[1]);
    double t_go = nrh / sqrt(vh[0] * vh[0] + vh[1] * vh[1]);
    double f = -(double)v0 / fmax(1e-3, nrh) * (1 - exp(-t_go / tau));
    double vt0 = f * rh[0], vt1 = f * rh[1];
    double vel = c->alfa * sqrt((s[3] - vt0) * (s[3] - vt0) + (s[4] - vt1) * (s[4] - vt1));
    double thr = c->beta * (double)u[1];
    double zeta = (double)s[2] - M_PI / 2;
    double attitude = c->gamma * (double)(fabs(zeta) > 2 * M_PI);
    double hint = c->delta * fmax(0.0, fabs(zeta) - M_PI / 2);
    double r = sqrt((double)s[0] * s[0] + (double)s[1] * s[1]);
    double v = sqrt((double)s[3] * s[3] + (double)s[4] * s[4]);
    int landing = (s[1] <= 1e-3) && (v < 15) && (r < c->landing_radius) && (fabs(zeta) < 0.2) &&
                  (fabsf(s[5]) < 0.2);
    double goal = c->kappa * landing;
    o->terms[0] = vel;
    o->terms[1] = thr;
    o->terms[2] = c->eta;
    o->terms[3] = attitude;
    o->terms[4] = hint;
    o->terms[5] = goal;
    o->reward = vel + thr + c->eta + attitude + hint + goal + (outside ? -50.0 : 0.0);
    /* _normalize_obs(state32) -> float64 obs (rocket_env.py:175, 209-210) */
    for (int i = 0; i < 7; ++i) o->obs[i] = (float)((double)s[i] / c->normalizer[i]);
}

/* _wrapTo2Pi, simulator.py:150-163 */
static double wrap_2pi(double a)
{
    const double p2 = 2.0 * M_PI;
    return fmod(fmod(a, p2) + p2, p2);
}

void ro_step(const ro_cfg* c, const float* ic, double t_in, const double* s_in, const float* a, ro_out* o)
{
    float u[3];
    ctrl k;
    memset(o, 0, sizeof(*o));
    denorm_action(c, a, u);
    make_ctrl(c, u, &k);
    const int n = c->model == 6 ? 14 : 7;
    const int idx = c->model == 6 ? 0 : 1;
    double y[NMAX];
    int nfev = 0;
    int status = c->integrator == RO_INT_EULER ? euler_step(c, &k, n, idx, s_in, y, &nfev)
                                               : solve_ivp_rk45(c, &k, n, idx, t_in, s_in, y, &nfev);
    if (c->model == 6) {
        /* _normalize_quaternion, simulator.py:250 */
        double nq = sqrt(y[6] * y[6] + y[7] * y[7] + y[8] * y[8] + y[9] * y[9]);
        for (int i = 6; i < 10; ++i) y[i] /= nq;
    } else {
        y[2] = wrap_2pi(y[2]);
    }
    memcpy(o->state, y, sizeof(double) * n);
    o->status = status;
    o->nfev = nfev;
    if (c->model == 6) env6_finish(c, ic, u, status, y, o);
    else env3_finish(c, ic, u, status, y, o);
}

void ro_step_batch(const ro_cfg* c, int64_t n, const float* ic, const double* t_in, const double* s_in,
                   const float* a, double* state_out, float* obs, double* reward, double* terms,
                   int32_t* done, int32_t* bounds_violation, int32_t* status, int32_t* nfev, int nthreads)
{
    const int ns = c->model == 6 ? 14 : 7;
    const int na = c->model == 6 ? 3 : 2;
    const int nt = c->model == 6 ? 5 : 6;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) if (nthreads != 1)
#endif
    for (int64_t i = 0; i < n; ++i) {
        ro_out o;
        ro_step(c, ic + i * ns, t_in[i], s_in + i * ns, a + i * na, &o);
        if (state_out) memcpy(state_out + i * ns, o.state, sizeof(double) * ns);
        if (obs) memcpy(obs + i * ns, o.obs, sizeof(float) * ns);
        if (reward) reward[i] = o.reward;
        if (terms) memcpy(terms + i * nt, o.terms, sizeof(double) * nt);
        if (done) done[i] = o.done;
        if (bounds_violation) bounds_violation[i] = o.bounds_violation;
        if (status) status[i] = o.status;
        if (nfev) nfev[i] = o.nfev;
    }
}

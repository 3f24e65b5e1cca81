/*
 * Rollout + MPC cost + argmin oracle in plain C, fp64 — TEST INFRASTRUCTURE ONLY.
 * Built by oracle/Makefile into oracle/_build/libmpcoracle.so; only tests/, smoke() and
 * bench.py's cpu_baseline leg load it. Compiled with -ffp-contract=off so every expression
 * rounds exactly as the reference's numpy/python fp64 evaluation does (left to right).
 *
 * Systems:
 *  0 cartpole_lin5  EulerForwardCartpole_virtual, linearised xdot_new
 *                   (scripts/inference/Cart_Diffusion_inference.py:122-130 constants,
 *                   :168-197 dynamics), cost = calMPCCost (:247-283) with Q,R,P of :37-41.
 *  1 cartpole_nl5   nonlinear Euler cart-pole (scripts/mpc_data_collecting/
 *                   nmpc_multi_process_collect_data.py:96-111 constants, :121-137 dynamics),
 *                   canonical cost (:143-172) with Q,R,P of :63-65, TS = 0.01.
 *  2 cartpole_zoh4  linear ZOH cart-pole, Ts = 0.1 (scripts/inference/Diffusion_MPC_Inference.py:39-84;
 *                   A_d/B_d = expm of the augmented matrix, SURVEY KAT6), canonical cost with
 *                   Q = diag(10,1,10,1), R = 1, P = diag(100,1,100,1) (:313-315, :357-371).
 *  3 double_int2d   BUILD-DEFINED 2D double integrator (no reference): x=[px,py,vx,vy], u=[ax,ay].
 *  4 pendulum       BUILD-DEFINED damped pendulum swing-up (no reference): x=[theta, omega], u=[tau].
 *  5 quadrotor12    BUILD-DEFINED 12-state rigid-body quadrotor (no reference).
 * Canonical cost (the reference's MPC objective, nmpc...py:158-172):
 *   J = q(x_0) ; for k = 0..H-2 { x_{k+1} = f(x_k,u_k); J += q(x_{k+1}) + r(u_k) } ;
 *   x_H = f(x_{H-1},u_{H-1}) ; J += p(x_H) + r(u_{H-1})
 * with q(x) = sum_j Q_j*(e_j*e_j) left to right, e = x - x_ref, r(u) = sum_i R_i*(u_i*u_i).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NX_MAX 12
#define NU_MAX 4

typedef struct {
    int nx, nu, cost_kind; /* cost_kind 0 canonical, 1 calMPCCost */
    double Q[NX_MAX], R[NU_MAX], P[NX_MAX], xref[NX_MAX];
} sys_info;

static const double PI_D = 3.141592653589793;

/* --- cart-pole constants, restated from the reference scripts --- */
/* Cart_Diffusion_inference.py:122-130 */
#define CP_MCAR 4.5
#define CP_MPOLE 0.12
#define CP_L 0.14
#define CP_K 0.5
#define CP_C 0.002
#define CP_G 9.81

static void cartpole_lin5_f(double dt, const double *x, double u, double *xn)
{
    const double I = (CP_MPOLE * (CP_L * CP_L)) / 3;  /* (m_pole*l_pendul**2)/3 */
    const double den = I * (CP_MCAR + CP_MPOLE) + (CP_L * CP_L) * CP_MPOLE * CP_MCAR;
    const double v1 = (CP_MCAR + CP_MPOLE) / den;
    const double v2 = (I + (CP_L * CP_L) * CP_MPOLE) / den;
    const double il = I + (CP_L * CP_L) * CP_MPOLE;
    const double lm = CP_L * CP_MPOLE;
    double xd[5];
    xd[0] = x[1];
    xd[1] = -CP_K * v2 * x[1] + (lm * lm) * CP_G * v2 / il * x[2] - lm * CP_C * v2 / il * x[3] + v2 * u;
    xd[2] = x[3];
    xd[3] = -CP_L * CP_MPOLE * CP_K * v1 / (CP_MCAR + CP_MPOLE) * x[1] + lm * CP_G * v1 * x[2]
            - CP_C * v1 * x[3] + lm * v1 / (CP_MCAR + CP_MPOLE) * u;
    xd[4] = -(2 / PI_D) * (x[2] - PI_D) * x[3];
    for (int i = 0; i < 5; ++i) xn[i] = x[i] + xd[i] * dt;
}

/* nmpc_multi_process_collect_data.py:96-111 */
static void cartpole_nl5_f(double dt, const double *x, double u, double *xn)
{
    const double M_CART = 2.0, M_POLE = 1.0, M_TOTAL = M_CART + M_POLE, L_POLE = 1.0, G = 9.81;
    const double MPLP = M_POLE * L_POLE, MPG = M_POLE * G, MTG = M_TOTAL * G, MTLP = M_TOTAL * G;
    const double s = sin(x[2]), c = cos(x[2]);
    const double dd = M_TOTAL - M_POLE * c;
    double xd[5];
    xd[0] = x[1];
    xd[1] = (MPLP * -s * (x[3] * x[3]) + MPG * s * c + u) / (dd * dd);
    xd[2] = x[3];
    xd[3] = (-MPLP * s * c * (x[3] * x[3]) - MTG * s - c * u) / (MTLP - MPLP * (c * c));
    xd[4] = -(2 / PI_D) * (x[2] - PI_D) * x[3];
    for (int i = 0; i < 5; ++i) xn[i] = x[i] + xd[i] * dt;
}

static const double ZOH_A[4][4] = {
    {1.0, 0.09949537483382852, 0.015327761653922887, 0.0005062874425049262},
    {0.0, 0.9897973187953647, 0.3136747477766333, 0.015327761653922889},
    {0.0, -0.0025546269423204816, 1.1535307602604814, 0.10506917464734186},
    {0.0, -0.05227912462943889, 3.144411358593294, 1.1535307602604812}};
static const double ZOH_B[4] = {0.010029501100503806, 0.20152218688018167, 0.025461888182787322,
                                0.5202366193520683};

static void cartpole_zoh4_f(const double *x, double u, double *xn)
{
    /* Diffusion_MPC_Inference.py:74-82: A[i,0]*x0 + A[i,1]*x1 + A[i,2]*x2 + A[i,3]*x3 + B[i]*u */
    for (int i = 0; i < 4; ++i)
        xn[i] = ZOH_A[i][0] * x[0] + ZOH_A[i][1] * x[1] + ZOH_A[i][2] * x[2] + ZOH_A[i][3] * x[3] + ZOH_B[i] * u;
}

static void double_int2d_f(const double *x, const double *u, double *xn)
{
    const double dt = 0.1, h = 0.5 * dt * dt;
    xn[0] = x[0] + dt * x[2] + h * u[0];
    xn[1] = x[1] + dt * x[3] + h * u[1];
    xn[2] = x[2] + dt * u[0];
    xn[3] = x[3] + dt * u[1];
}

static void pendulum_f(const double *x, double u, double *xn)
{
    const double dt = 0.05, g_l = 9.81 / 1.0, damp = 0.1, inv_ml2 = 1.0 / (1.0 * 1.0 * 1.0);
    xn[0] = x[0] + dt * x[1];
    xn[1] = x[1] + dt * (-g_l * sin(x[0]) - damp * x[1] + inv_ml2 * u);
}

static void quadrotor12_f(const double *x, const double *u, double *xn)
{
    const double dt = 0.02, m = 1.0, g = 9.81, Ix = 0.01, Iy = 0.01, Iz = 0.02;
    const double sph = sin(x[3]), cph = cos(x[3]), sth = sin(x[4]), cth = cos(x[4]);
    const double sps = sin(x[5]), cps = cos(x[5]);
    const double f_m = (m * g + u[0]) / m;
    double xd[12];
    xd[0] = x[6];
    xd[1] = x[7];
    xd[2] = x[8];
    xd[3] = x[9] + (x[10] * sph + x[11] * cph) * (sth / cth);
    xd[4] = x[10] * cph - x[11] * sph;
    xd[5] = (x[10] * sph + x[11] * cph) / cth;
    xd[6] = f_m * (cph * sth * cps + sph * sps);
    xd[7] = f_m * (cph * sth * sps - sph * cps);
    xd[8] = f_m * (cph * cth) - g;
    xd[9] = ((Iy - Iz) * x[10] * x[11] + u[1]) / Ix;
    xd[10] = ((Iz - Ix) * x[9] * x[11] + u[2]) / Iy;
    xd[11] = ((Ix - Iy) * x[9] * x[10] + u[3]) / Iz;
    for (int i = 0; i < 12; ++i) xn[i] = x[i] + dt * xd[i];
}

static int get_info(int system, sys_info *si)
{
    memset(si, 0, sizeof(*si));
    switch (system) {
    case 0: { /* Cart_Diffusion_inference.py:37-41 */
        const double q[5] = {0.01, 0.01, 0, 0.001, 1000.0};
        si->nx = 5; si->nu = 1; si->cost_kind = 1;
        for (int i = 0; i < 5; ++i) { si->Q[i] = q[i]; si->P[i] = q[i]; }
        si->R[0] = 0.1;
        return 0; }
    case 1: { /* nmpc_multi_process_collect_data.py:63-65 */
        const double q[5] = {0.01, 0.01, 0, 0.01, 1000.0}, p[5] = {0.01, 0.1, 0, 0.1, 1000.0};
        si->nx = 5; si->nu = 1;
        for (int i = 0; i < 5; ++i) { si->Q[i] = q[i]; si->P[i] = p[i]; }
        si->R[0] = 0.001;
        return 0; }
    case 2: { const double q[4] = {10, 1, 10, 1}, p[4] = {100, 1, 100, 1};
        si->nx = 4; si->nu = 1;
        for (int i = 0; i < 4; ++i) { si->Q[i] = q[i]; si->P[i] = p[i]; }
        si->R[0] = 1.0;
        return 0; }
    case 3: { const double q[4] = {1, 1, 0.1, 0.1}, p[4] = {10, 10, 1, 1};
        si->nx = 4; si->nu = 2;
        for (int i = 0; i < 4; ++i) { si->Q[i] = q[i]; si->P[i] = p[i]; }
        si->R[0] = si->R[1] = 0.01;
        return 0; }
    case 4: si->nx = 2; si->nu = 1;
        si->Q[0] = 10; si->Q[1] = 0.1; si->P[0] = 100; si->P[1] = 1; si->R[0] = 0.01; si->xref[0] = PI_D;
        return 0;
    case 5: { const double q[12] = {10, 10, 10, 1, 1, 1, 1, 1, 1, 0.1, 0.1, 0.1};
        const double r[4] = {0.1, 1, 1, 1};
        si->nx = 12; si->nu = 4;
        for (int i = 0; i < 12; ++i) { si->Q[i] = q[i]; si->P[i] = 10 * q[i]; }
        for (int i = 0; i < 4; ++i) si->R[i] = r[i];
        return 0; }
    default: return -1;
    }
}

static void step(int system, const double *x, const double *u, double *xn)
{
    switch (system) {
    case 0: cartpole_lin5_f(0.01, x, u[0], xn); break;
    case 1: cartpole_nl5_f(0.01, x, u[0], xn); break;
    case 2: cartpole_zoh4_f(x, u[0], xn); break;
    case 3: double_int2d_f(x, u, xn); break;
    case 4: pendulum_f(x, u[0], xn); break;
    case 5: quadrotor12_f(x, u, xn); break;
    }
}

static double quad(const double *w, const double *x, const double *ref, int n)
{
    double s = 0.0;
    for (int j = 0; j < n; ++j) { const double e = x[j] - ref[j]; s = s + w[j] * (e * e); }
    return s;
}

/* calMPCCost, Cart_Diffusion_inference.py:247-283 (num_u = 1: the batch axis of u_hor) */
static double cal_mpc_cost(const sys_info *si, int system, const double *x0, const double *u, int H)
{
    double cost = 0.0, xc[NX_MAX], xn[NX_MAX];
    for (int i = 0; i < si->nx; ++i) cost = cost + si->Q[i] * (x0[i] * x0[i]);
    cost = cost + si->R[0] * (u[0] * u[0]);
    memcpy(xc, x0, sizeof(double) * si->nx);
    memcpy(xn, x0, sizeof(double) * si->nx);
    double ucur = u[0];
    for (int i = 1; i < H - 1; ++i) {
        step(system, xc, &ucur, xn);
        const double unext = u[i];
        for (int j = 1; j < si->nx; ++j) cost = cost + si->Q[j] * (xn[j] * xn[j]);
        cost = cost + si->R[0] * (unext * unext);
        ucur = unext;
        memcpy(xc, xn, sizeof(double) * si->nx);
    }
    for (int i = 0; i < si->nx; ++i) cost = cost + si->P[i] * (xn[i] * xn[i]);
    return cost;
}

static double canonical_cost(const sys_info *si, int system, const double *x0, const double *u, int H)
{
    double xc[NX_MAX], xn[NX_MAX];
    const int nx = si->nx, nu = si->nu;
    double J = quad(si->Q, x0, si->xref, nx);
    memcpy(xc, x0, sizeof(double) * nx);
    for (int k = 0; k < H; ++k) {
        step(system, xc, u + (size_t)k * nu, xn);
        const double zero[NU_MAX] = {0, 0, 0, 0};
        const double sx = (k < H - 1) ? quad(si->Q, xn, si->xref, nx) : quad(si->P, xn, si->xref, nx);
        const double su = quad(si->R, u + (size_t)k * nu, zero, nu);
        J = J + (sx + su);
        memcpy(xc, xn, sizeof(double) * nx);
    }
    return J;
}

int oracle_system_info(int system, int *nx, int *nu, int *cost_kind, double *Q, double *R, double *P, double *xref)
{
    sys_info si;
    if (get_info(system, &si)) return -1;
    *nx = si.nx; *nu = si.nu; *cost_kind = si.cost_kind;
    memcpy(Q, si.Q, sizeof(si.Q)); memcpy(R, si.R, sizeof(si.R));
    memcpy(P, si.P, sizeof(si.P)); memcpy(xref, si.xref, sizeof(si.xref));
    return 0;
}

/* One candidate step of the dynamics, exposed for tests. */
int oracle_step(int system, const double *x, const double *u, double *xn)
{
    sys_info si;
    if (get_info(system, &si)) return -1;
    step(system, x, u, xn);
    return 0;
}

/* u: [B, H, nu] fp64 (already unnormalised), cost: [B] */
int oracle_rollout_cost(int system, const double *x0, const double *u, int64_t B, int H, double *cost)
{
    sys_info si;
    if (get_info(system, &si) || H < 2) return -1;
    for (int64_t b = 0; b < B; ++b) {
        const double *ub = u + (size_t)b * H * si.nu;
        cost[b] = si.cost_kind == 1 ? cal_mpc_cost(&si, system, x0, ub, H) : canonical_cost(&si, system, x0, ub, H);
    }
    return 0;
}

/* argmin with NaN treated as +inf and ties resolved to the lowest index */
int64_t oracle_argmin(const double *cost, int64_t n)
{
    int64_t best = -1;
    double bv = INFINITY;
    for (int64_t i = 0; i < n; ++i) {
        const double v = isnan(cost[i]) ? INFINITY : cost[i];
        if (best < 0 || v < bv) { bv = v; best = i; }
    }
    return best;
}

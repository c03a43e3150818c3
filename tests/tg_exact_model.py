"""Exact enumeration of the two-group semi-Markov model on tiny chains (TEST
INFRASTRUCTURE ONLY).

An independent restatement, in numpy/scipy float64, of the reference's MODEL --
not of its particle filter -- written from the reference files directly and
sharing nothing with oracle/ or include/ (no tables, no arithmetic contract):

- parameters: Beta(alpha, beta) by moments (case_control_regime_model.py:19-23);
  control transition matrix = softmax(theta blocks) with -inf diagonal
  (run_inference_two_groups.py:76-89, case_control_regime_model.py:90-94);
  merge/split matrix softmax(P_softmax_merged) (run_inference_two_groups.py:
  164-167); the parameter VALUES rounded to float32 as the reference's
  tf.Variables hold them, the arithmetic in float64;
- emission: sum over samples of scipy.stats.betabinom.logpmf
  (case_control_regime_model.py:197-231), n = 0 terms exactly 0;
- hazard: rho(d) = NB_pmf(d - u) / P(X > d - u - 1) with scipy.stats.nbinom
  (tfd.NegativeBinomial(total_count=kappa, probs=omega): pmf = C(x+k-1, x)
  (1-omega)^k omega^x, i.e. scipy p = 1 - omega), 0 below u, the survival 1 at
  d == u, 0.1 when not finite (case_control_regime_model.py:111-168); the
  survival is log1p(-cdf) with the cdf rounded to float32, as TFP holds it;
- transition: merged switch only if min(d_ctrl, d_case) >= u (:80-87); control
  (case_control_distributions.py:138-151); case, four branches (:246-291);
- t = 0: the transition from the phantom (m = 1, d = 0, r_ph) with rho = 1
  (case_control_regime_model.py:234-244, :164-167 step == 0 rows).

The forward / backward recursions run over the explicit reachable state set
(m, d_c, r_c, d_k, r_k) -- successors are found by trying every (m', d' in
{1, d + 1}, r') for both groups, never by the reference's proposal mapping --
so the exact log marginal likelihood, filter and smoothing marginals and
pairwise smoothing marginals given the phantom regime are available.
"""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np
from scipy import stats
from scipy.special import logsumexp

f32 = lambda x: float(np.float32(x))  # noqa: E731


class ExactModel:
    def __init__(self, K, mu, sigma, theta, u=3, omega_case=0.8, merge_log_prob=math.log(0.1), split_prob=0.01,
                 kappa=2.0, case_uniform_sizes=None):
        self.K, self.u = K, u
        # sizes of the case transition's uniform regime draws per branch (2, 3, 4);
        # None = the reference's allowed sets. Tests override one of them to show
        # that the log Z comparison would catch a wrong normaliser.
        self.case_uniform_sizes = case_uniform_sizes or {}
        mu = np.array([f32(v) for v in mu])
        sg = np.array([f32(v) for v in sigma])
        nu = mu * (1 - mu) / sg ** 2 - 1
        self.alpha, self.beta = mu * nu, (1 - mu) * nu
        theta = np.asarray(theta, np.float64)
        # control transition matrix (row r: softmax over r' != r of theta's block r)
        self.lPc = np.full((K, K), -np.inf)
        i = 0
        for r in range(K):
            blk = theta[i:i + K - 1]
            i += K - 1
            v = np.array([f32(x) for x in blk - logsumexp(blk)])
            cols = [c for c in range(K) if c != r]
            self.lPc[r, cols] = v - logsumexp(v)
        om_logit = theta[len(theta) - K:]
        self.om_ctrl = np.array([f32(1.0 / (1.0 + math.exp(-f32(x)))) for x in om_logit])
        self.om_case = np.full(K, f32(omega_case))
        self.kappa = f32(kappa)
        v0 = np.array([f32(math.log(1 - math.exp(merge_log_prob))), f32(merge_log_prob)])
        v1 = np.array([f32(math.log(split_prob)), f32(math.log(1 - split_prob))])
        self.lPm = np.array([v0 - logsumexp(v0), v1 - logsumexp(v1)])  # [m][m']
        self._rho = {}
        self._succ = {}

    # ------------------------------------------------------------ pieces
    def rho(self, g, r, d):
        key = (g, r, d)
        if key not in self._rho:
            if d < self.u:
                v = 0.0
            else:
                om = (self.om_case if g else self.om_ctrl)[r]
                nb = stats.nbinom(self.kappa, 1.0 - om)
                lh = nb.logpmf(d - self.u)
                # TFP's float32 survival: log1p(-cdf) with the cdf held in float32
                ls = 0.0 if d == self.u else math.log1p(-f32(nb.cdf(d - self.u - 1)))
                v = math.exp(lh - ls) if lh > -np.inf else 0.0
                if not math.isfinite(v):
                    v = 0.1
            self._rho[key] = v
        return self._rho[key]

    def emission(self, meth_c, tot_c, meth_k, tot_k):
        """log g_t for control regime r and case regime r': [T][2K]."""
        T = tot_c.shape[0]
        E = np.zeros((T, 2 * self.K))
        for g, (y, n) in enumerate(((meth_c, tot_c), (meth_k, tot_k))):
            for r in range(self.K):
                lp = stats.betabinom.logpmf(y.astype(np.int64), n.astype(np.int64), self.alpha[r], self.beta[r])
                lp = np.where(n == 0, 0.0, lp)
                E[:, g * self.K + r] = lp.sum(1)
        return E

    def log_trans(self, x, y):
        """log f_t(y | x) for t >= 1; states (m, dc, rc, dk, rk)."""
        m, dc, rc, dk, rk = x
        m2, dc2, rc2, dk2, rk2 = y
        K = self.K
        # merged state (case_control_regime_model.py:80-87)
        if min(dk, dc) >= self.u:
            lm = self.lPm[m, m2]
        else:
            lm = 0.0 if m2 == m else -np.inf
        # control (case_control_distributions.py:138-151)
        rho_c = self.rho(0, rc, dc)
        if dc2 == 1:
            lc = _log(rho_c) + self.lPc[rc, rc2]
        else:
            lc = _log(1 - rho_c) if (dc2 == dc + 1 and rc2 == rc) else -np.inf
        # case (case_control_distributions.py:246-291)
        branch = self.case_branch(x, y)
        sz = lambda allowed: self.case_uniform_sizes.get(branch, len(allowed))  # noqa: E731
        if branch == 1:
            lk = 0.0 if (rk2 == rc2 and dk2 == dc2) else -np.inf
        elif branch == 2:
            allowed = [r for r in range(K) if r != rc2]
            lk = -math.log(sz(allowed)) if (dk2 == 1 and rk2 in allowed) else -np.inf
        elif branch == 3:
            allowed = [r for r in range(K) if r != rc2 and r != rk]
            lk = -math.log(sz(allowed)) if (dk2 == 1 and rk2 in allowed and allowed) else -np.inf
        else:
            rho_k = self.rho(1, rk, dk)
            if dk2 == 1:
                allowed = [r for r in range(K) if r != rc2 and r != rk]
                lk = _log(rho_k) - math.log(sz(allowed)) if (rk2 in allowed) else -np.inf
            else:
                lk = _log(1 - rho_k) if (dk2 == dk + 1 and rk2 == rk) else -np.inf
        return lm + lc + lk

    @staticmethod
    def case_branch(x, y):
        """Which of the four branches of CaseStateTransition._log_prob
        (case_control_distributions.py:246-291) scores the case part of x -> y:
        1 merged next state; 2 a merged ancestor splits while the control
        continues (case regime uniform over r != r_c', 1/(K-1)); 3 a split
        ancestor whose control moves onto the case regime (uniform over
        r not in {r_c', r_k}, here 1/(K-1)); 4 otherwise (hazard rho_k, a change
        uniform over r not in {r_c', r_k}: 1/(K-2) when r_c' != r_k)."""
        m, _, _, _, rk = x
        m2, dc2, rc2, _, _ = y
        if m2 == 1:
            return 1
        if m == 1 and dc2 != 1:
            return 2
        if rc2 == rk and m == 0:
            return 3
        return 4

    def successors(self, x):
        """[(y, log f(y | x))] over every y with a finite transition density
        (memoised: the transitions do not depend on the phantom regime)."""
        got = self._succ.get(x)
        if got is None:
            got = self._succ[x] = list(self._successors(x))
        return got

    def _successors(self, x):
        m, dc, rc, dk, rk = x
        for m2 in (0, 1):
            for dc2 in (1, dc + 1):
                for rc2 in range(self.K):
                    for dk2 in sorted({1, dk + 1, dc2}):
                        for rk2 in range(self.K):
                            y = (m2, dc2, rc2, dk2, rk2)
                            lf = self.log_trans(x, y)
                            if lf > -np.inf:
                                yield y, lf

    def initial(self, r_ph):
        """t = 0 prior: the transition from the phantom (1, 0, r_ph, 0, r_ph) at
        step 0 (rho = 1, merged row [0, 1], case deterministic)."""
        return {(1, 1, i, 1, i): self.lPc[r_ph, i] for i in range(self.K) if self.lPc[r_ph, i] > -np.inf}

    # -------------------------------------------------------- recursions
    def log_z(self, E, r_ph):
        """The exact log marginal likelihood given the phantom regime alone (the
        forward recursion of forward_backward, without the smoother)."""
        K = self.K
        lg = lambda t, x: E[t, x[2]] + E[t, K + x[4]]  # noqa: E731
        alpha = {x: v + lg(0, x) for x, v in self.initial(r_ph).items()}
        for t in range(1, E.shape[0]):
            nxt = defaultdict(list)
            for x, a in alpha.items():
                for y, lf in self.successors(x):
                    nxt[y].append(a + lf)
            alpha = {y: logsumexp(v) + lg(t, y) for y, v in nxt.items()}
        return logsumexp(list(alpha.values()))

    def forward_backward(self, E, r_ph):
        """Exact log Z and the filter / smoothing marginals given the phantom
        regime. Returns (log_z, alphas, smooth, pair) with alphas[t]: {x: log
        alpha_t(x)}, smooth[t]: {x: p(x_t | y)}, pair[t]: {(x, y): p(x_t, x_{t+1} | y)}."""
        K = self.K
        T = E.shape[0]
        lg = lambda t, x: E[t, x[2]] + E[t, K + x[4]]  # noqa: E731
        alphas = [{x: v + lg(0, x) for x, v in self.initial(r_ph).items()}]
        trans = []
        for t in range(1, T):
            nxt = defaultdict(list)
            tt = {}
            for x, a in alphas[-1].items():
                succ = list(self.successors(x))
                tt[x] = succ
                for y, lf in succ:
                    nxt[y].append(a + lf)
            alphas.append({y: logsumexp(v) + lg(t, y) for y, v in nxt.items()})
            trans.append(tt)
        log_z = logsumexp(list(alphas[-1].values()))
        betas = [None] * T
        betas[T - 1] = {x: 0.0 for x in alphas[T - 1]}
        for t in range(T - 2, -1, -1):
            b = {}
            for x in alphas[t]:
                b[x] = logsumexp([lf + lg(t + 1, y) + betas[t + 1][y] for y, lf in trans[t][x]])
            betas[t] = b
        smooth = [{x: math.exp(alphas[t][x] + betas[t][x] - log_z) for x in alphas[t]} for t in range(T)]
        pair = []
        for t in range(T - 1):
            d = {}
            for x in alphas[t]:
                for y, lf in trans[t][x]:
                    d[(x, y)] = math.exp(alphas[t][x] + lf + lg(t + 1, y) + betas[t + 1][y] - log_z)
            pair.append(d)
        return log_z, alphas, smooth, pair


def _log(v):
    return math.log(v) if v > 0 else -np.inf


def unpack(s: int):
    """Packed particle state of the oracle / kernels (include/hyg_arith.h)."""
    s = int(s)
    return ((s >> 60) & 1, s & 0xFFFFFF, (s >> 48) & 63, (s >> 24) & 0xFFFFFF, (s >> 54) & 63)


def phantom_regime(oracle, seed: int, chain_id: int, K: int) -> int:
    """r_ph of a chain: Philox stream 1 at (step 0, index 0), scaled to [0, K)
    (the uniform the oracle consumes for case_control_distributions.py:67-74)."""
    import ctypes

    out = (ctypes.c_uint64 * 4)()
    oracle.lib().oracle_philox(1, 0, 0, 0, seed, chain_id, ctypes.addressof(out))
    return (int(out[0]) * K) >> 64

"""Host-side mirror of the reference's two-group inference interface.

Reference (src/two_group): the model is built as
    CaseControlRegimeModel(n_methylation_regimes, mu, sigma, P_softmax_control,
        P_softmax_merged, omega_inv_logit_control, omega_inv_logit_case,
        minimum_duration, kappa_control, kappa_case, n_total_reads_control,
        n_total_reads_case)                      (hygeia/case_control_regime_model.py:47-74)
from the CLI flags and the single-group theta (run_inference_two_groups.py:110-167),
and inference is
    filter_and_smoother_algorithm.run(observations, ..., num_particles,
        num_resampled_ancestors, optimal_resampling=True, num_simulations)
      -> (BackwardSimulationResults(step, particle={'merged_state', 'control_state',
          'case_state'}), final_unnormalized_log_weights)      (filter_and_smoother_algorithm.py:38-138)

Here `CaseControlModel` holds the same parameters (as a C-ABI model handle with
its tables on the GPU) and `run()` has the same meaning and return structure.
Every computation runs in the HIP kernels of libhygeia_amd.so; there is no CPU
fallback (without a HIP device the library raises HygError(HYG_EDEVICE)).
"""
from __future__ import annotations

import collections
import ctypes as C
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

BackwardSimulationResults = collections.namedtuple("BackwardSimulationResults", ["step", "particle"])


def theta_to_matrix(theta: Sequence[float], K: int) -> Tuple[np.ndarray, np.ndarray]:
    """get_estimated_control_group_param (run_inference_two_groups.py:76-89):
    returns (log P_ctrl [K,K] with -inf diagonal, omega_logit_control [K])."""
    p = np.zeros((K, K))
    i = 0
    for r in range(K):
        for r1 in range(K):
            if r != r1:
                p[r, r1] = math.exp(theta[i])
                i += 1
        p[r, :] /= p[r, :].sum()
    with np.errstate(divide="ignore"):
        return np.log(p), np.asarray(theta[-K:], dtype=np.float64)


def uniform_theta(K: int, omega: float = 0.8) -> np.ndarray:
    return np.concatenate([np.zeros(K * (K - 1)), np.full(K, math.log(omega / (1.0 - omega)))])


class CaseControlModel:
    """Parameters of CaseControlRegimeModel + the proposal sizes, as a C-ABI model."""

    def __init__(self, mu: Sequence[float], sigma: Sequence[float], theta: Sequence[float],
                 minimum_duration: int = 3, omega_case: float = 0.8, merge_log_prob: float = math.log(0.1),
                 split_prob: float = 0.01, num_resampled_ancestors: int = 50, num_samples_backward: int = 25,
                 kappa_control: float = 2.0, kappa_case: float = 2.0, max_total_reads: int = 1023,
                 max_duration: int = 110000, optimal_resampling: bool = True, multinomial: bool = False):
        self.params = _lib.make_params(mu, sigma, theta, minimum_duration, num_resampled_ancestors,
                                       num_samples_backward, omega_case, merge_log_prob, split_prob,
                                       kappa_control, kappa_case, optimal_resampling, multinomial)
        self.n_regimes = len(mu)
        self.num_resampled_ancestors = int(num_resampled_ancestors)
        self.num_samples_backward = int(num_samples_backward)
        self.max_total_reads = int(max_total_reads)
        self.max_duration = int(max_duration)
        L = _lib.load()
        h = C.c_void_p()
        _lib.check(L.hyg_tg_model_create(C.byref(self.params), self.max_total_reads, self.max_duration, C.byref(h)))
        self._h = h

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def num_particles(self) -> int:
        """N_max = M (2K + K^2) (run_inference_two_groups.py:263)."""
        return int(_lib.load().hyg_tg_num_particles(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.load().hyg_tg_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _u16(a) -> np.ndarray:
    a = np.asarray(a)
    if a.ndim == 1:
        a = a[:, None]
    if np.any(a < 0) or np.any(a > 65535) or np.any(np.floor(a) != a):
        raise ValueError("read counts must be integers in [0, 65535]")
    return np.ascontiguousarray(a, dtype=np.uint16)


def run(observations: Dict[str, np.ndarray], n_total_reads: Dict[str, np.ndarray], model: CaseControlModel,
        seed: int, chain_id: int = 0):
    """filter_and_smoother_algorithm.run for the CaseControlRegimeModel: particle
    filter with optimal finite-state resampling + backward simulation of
    num_samples_backward trajectories.

    observations / n_total_reads: {'control': [T,S_c], 'case': [T,S_k]} methylated
    and total read counts. Returns (BackwardSimulationResults, final weights
    [N_max], extras) with extras = {'split_probs', 'regime_probs', 'log_z'} the
    posterior means of run_inference_two_groups.py:233-240, 289-296.
    """
    mc, tc = _u16(observations["control"]), _u16(n_total_reads["control"])
    mk, tk = _u16(observations["case"]), _u16(n_total_reads["case"])
    T = tc.shape[0]
    if mc.shape != tc.shape or mk.shape != tk.shape or tk.shape[0] != T:
        raise ValueError("inconsistent count shapes")
    if T > model.max_duration:
        raise ValueError(f"{T} sites exceed the model's max_duration {model.max_duration}")
    K, B, N = model.n_regimes, model.num_samples_backward, model.num_particles
    merged = np.empty((T, B), np.int16)
    control = np.empty((T, B, 2), np.int16)
    case = np.empty((T, B, 2), np.int16)
    split = np.empty(T, np.float32)
    regime = np.empty((T, 2 * K), np.float32)
    final_w = np.empty(N, np.float64)
    log_z = C.c_double(0.0)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _lib.check(_lib.load().hyg_tg_run_chain_host(
        model.handle, p(mc), p(tc), mc.shape[1], p(mk), p(tk), mk.shape[1], T, int(seed), int(chain_id),
        p(merged), p(control), p(case), p(split), p(regime), C.byref(log_z), p(final_w)))
    res = BackwardSimulationResults(step=np.arange(T), particle={
        "merged_state": merged, "control_state": control, "case_state": case})
    return res, final_w, {"split_probs": split, "regime_probs": regime, "log_z": log_z.value}


def run_chains_host(observations: Dict[str, np.ndarray], n_total_reads: Dict[str, np.ndarray],
                    model: CaseControlModel, chains: List[Tuple[int, int, int, int, int]], n_out_rows: int,
                    final_weights: bool = False) -> Dict[str, np.ndarray]:
    """Many chains in one launch from host arrays (hyg_tg_run_chains_host), with
    no torch: `hygeia infer_many`'s every (batch, seed) task of a chromosome.
    chains: (site_begin, n_sites, seed, chain_id, out_begin) over the count rows
    and the output rows. Returns host arrays: merged [R,B], control / case
    [R,B,2], split_probs [R], regime_probs [R,2K], log_z / status [n_chains]
    (and final_w [n_chains, N_max]); each chain's rows are those of run()."""
    mc, tc = _u16(observations["control"]), _u16(n_total_reads["control"])
    mk, tk = _u16(observations["case"]), _u16(n_total_reads["case"])
    T = tc.shape[0]
    if mc.shape != tc.shape or mk.shape != tk.shape or tk.shape[0] != T:
        raise ValueError("inconsistent count shapes")
    if not chains:
        raise ValueError("no chains to run")
    n_rows = int(n_out_rows)
    spans = sorted((int(c[4]), int(c[4]) + int(c[1])) for c in chains)
    if spans[0][0] < 0 or spans[-1][1] > n_rows or any(a[1] > b[0] for a, b in zip(spans, spans[1:])):
        raise ValueError("chains' output rows [out_begin, out_begin + n_sites) must be disjoint and inside "
                         f"[0, {n_rows})")
    if max(int(c[1]) for c in chains) > model.max_duration:
        raise ValueError(f"a chain exceeds the model's max_duration {model.max_duration}")
    arr = (_lib.TgChain * len(chains))()
    for i, (site_begin, n_sites, seed, chain_id, out_begin) in enumerate(chains):
        arr[i].site_begin, arr[i].n_sites = int(site_begin), int(n_sites)
        arr[i].seed, arr[i].chain_id, arr[i].out_begin = int(seed), int(chain_id), int(out_begin)
    K, B, R, n = model.n_regimes, model.num_samples_backward, int(n_out_rows), len(chains)
    out = {"merged": np.empty((R, B), np.int16), "control": np.empty((R, B, 2), np.int16),
           "case": np.empty((R, B, 2), np.int16), "split_probs": np.empty(R, np.float32),
           "regime_probs": np.empty((R, 2 * K), np.float32), "log_z": np.empty(n, np.float64),
           "status": np.empty(n, np.int32)}
    if final_weights:
        out["final_w"] = np.empty((n, model.num_particles), np.float64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _lib.check(_lib.load().hyg_tg_run_chains_host(
        model.handle, p(mc), p(tc), mc.shape[1], p(mk), p(tk), mk.shape[1], T, arr, n, R, p(out["merged"]),
        p(out["control"]), p(out["case"]), p(out["split_probs"]), p(out["regime_probs"]), p(out["log_z"]),
        p(out["final_w"]) if final_weights else None, p(out["status"])))
    return out


class DeviceChains:
    """Batched device-resident execution of many chains (the bench and the
    multi-chain driver): emission table, history workspace and outputs are
    torch tensors on the current HIP device; kernels go to `stream`.
    `workspace` (uint8 tensor) lets batches that run one after another on one
    stream share the forward->backward history buffer."""

    @staticmethod
    def workspace_bytes(model: CaseControlModel, chains) -> int:
        return int(_lib.load().hyg_tg_workspace_bytes(model.handle, len(chains), sum(int(c[1]) for c in chains)))

    def __init__(self, model: CaseControlModel, chains: List[Tuple[int, int, int, int, int]], n_out_rows: int,
                 device=None, final_weights: bool = False, workspace=None):
        import torch

        if _lib.load() is not None and not _lib.loaded_with_torch():
            raise RuntimeError("the HIP library was loaded without torch (import_torch=False): torch's HIP "
                               "runtime must initialise first for device-tensor chains")

        self.torch = torch
        self.model = model
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        K, B = model.n_regimes, model.num_samples_backward
        self.chains = chains
        arr = (_lib.TgChain * len(chains))()
        total = 0
        for i, (site_begin, n_sites, seed, chain_id, out_begin) in enumerate(chains):
            arr[i].site_begin, arr[i].n_sites = int(site_begin), int(n_sites)
            arr[i].seed, arr[i].chain_id, arr[i].out_begin = int(seed), int(chain_id), int(out_begin)
            total += int(n_sites)
        self._arr = arr
        L = _lib.load()
        self.ws_bytes = int(L.hyg_tg_workspace_bytes(model.handle, len(chains), total))
        dev = self.device
        if workspace is not None:  # shared with other DeviceChains run one after another on one stream
            if workspace.numel() < self.ws_bytes or workspace.dtype != torch.uint8:
                raise ValueError(f"workspace of {workspace.numel()} bytes < {self.ws_bytes} needed")
            self.ws = workspace
        else:
            self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        self.merged = torch.empty((n_out_rows, B), dtype=torch.int16, device=dev)
        self.control = torch.empty((n_out_rows, B, 2), dtype=torch.int16, device=dev)
        self.case = torch.empty((n_out_rows, B, 2), dtype=torch.int16, device=dev)
        self.split_probs = torch.empty(n_out_rows, dtype=torch.float32, device=dev)
        self.regime_probs = torch.empty((n_out_rows, 2 * K), dtype=torch.float32, device=dev)
        self.log_z = torch.empty(len(chains), dtype=torch.float64, device=dev)
        self.status = torch.zeros(len(chains), dtype=torch.int32, device=dev)
        self.final_w = (torch.empty((len(chains), model.num_particles), dtype=torch.float64, device=dev)
                        if final_weights else None)
        self._out = _lib.TgOutputs(self.merged.data_ptr(), self.control.data_ptr(), self.case.data_ptr(),
                                   self.split_probs.data_ptr(), self.regime_probs.data_ptr(), self.log_z.data_ptr(),
                                   self.final_w.data_ptr() if self.final_w is not None else None,
                                   self.status.data_ptr())

    def emission(self, meth_c, tot_c, meth_k, tot_k, E=None, stream=None):
        """Beta-Binomial emission table [n_sites, 2K] f64 from device uint16 counts."""
        torch = self.torch
        T = tot_c.shape[0]
        if E is None:
            E = torch.empty((T, 2 * self.model.n_regimes), dtype=torch.float64, device=self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.load().hyg_tg_emission(self.model.handle, meth_c.data_ptr(), tot_c.data_ptr(),
                                               tot_c.shape[1], meth_k.data_ptr(), tot_k.data_ptr(), tot_k.shape[1],
                                               T, E.data_ptr(), C.c_void_p(s)))
        return E

    def run(self, E, stream=None) -> None:
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.load().hyg_tg_run_chains(self.model.handle, self._arr, len(self.chains), E.data_ptr(),
                                                 self.ws.data_ptr(), self.ws_bytes, C.byref(self._out),
                                                 C.c_void_p(s)))

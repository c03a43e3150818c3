"""Node-local chain server for concurrent `hygeia infer` tasks.

The reference's Nextflow module starts one `hygeia infer` process per
(chromosome, segment, seed) (modules/two_group/4_infer.nf:28,42-48), many at
once on a node (nextflow.config:17-21). Each process alone launches one chain:
one workgroup on a 256-CU GPU and a HIP runtime of its own, and beyond about
eight processes the GPU's hardware scheduler time-slices their queues
(a chain takes 1.75 s alone, 1.8 s beside 7 other task processes
and 2.5 s, up to 3.7 s, beside 15). One launch of the same 16 chains takes
1.86 s.

So an operator may run `hygeia serve` on the node (in the foreground, under
the node's service manager or beside the pipeline; `hygeia serve --stop` ends
it). While it runs, each `hygeia infer` task hands its chain to it: the task
still parses its inputs and writes its result files itself (the module's
contract is unchanged), but the chain runs in the server, which puts every
chain that is waiting when a GPU comes free into ONE launch
(hyg_tg_run_chains_host, the launch `hygeia infer_many` uses). A chain's
outputs do not depend on the launch it runs in (GPU tests), so the files are
those of the stand-alone task. Tasks never start a server themselves.

A task uses the server whose socket answers in the device lock directory
($HYGEIA_DEVICE_LOCK_DIR, else parallel.default_lock_dir: under Nextflow the
run's workDir, which every task container mounts); $HYGEIA_SERVER=0 makes it
ignore a server. A task that cannot reach one runs its chain itself.

Wire format (UNIX stream socket, one request per connection): an 8-byte
little-endian header length, a JSON header naming the sizes of the binary
buffers that follow, then the buffers.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket
import struct
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

MODE_VAR = "HYGEIA_SERVER"  # "0": tasks ignore a running server
SOCK_NAME = "hygeia_amd.server.sock"
IDLE_S = 0.0  # 0: run until stopped
MAX_HEADER = 1 << 20
SERVER_FAULT = 1  # reply code of a failure of the server itself (not of the chain): the task runs the chain itself


class ServerUnavailable(RuntimeError):
    """No server could be reached (the caller runs the chain itself)."""


# ----------------------------------------------------------------- framing
def send_msg(sock: socket.socket, header: dict, bufs: Sequence = ()) -> None:
    views = [memoryview(b).cast("B") for b in bufs]
    h = json.dumps(dict(header, sizes=[v.nbytes for v in views])).encode()
    sock.sendall(struct.pack("<Q", len(h)) + h)
    for v in views:
        sock.sendall(v)


def _recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("connection closed mid-message")
        got += k
    return buf


def recv_msg(sock: socket.socket) -> Tuple[dict, List[bytearray]]:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    if n > MAX_HEADER:
        raise ConnectionError("oversized header")
    header = json.loads(_recv_exact(sock, n).decode())
    return header, [_recv_exact(sock, int(s)) for s in header.get("sizes", [])]


# ------------------------------------------------------------ where / when
def socket_path(lock_dir: str) -> str:
    """The server socket in the lock directory; a UNIX socket path is limited
    to 107 bytes, so a longer one moves to /tmp under a digest of the directory."""
    p = os.path.join(lock_dir, SOCK_NAME)
    if len(p.encode()) < 100:
        return p
    return os.path.join("/tmp", f"hygeia_amd.{hashlib.sha1(lock_dir.encode()).hexdigest()[:16]}.sock")


def lock_dir(environ=None, cwd: str = None) -> Tuple[str, str]:
    from . import parallel

    env = os.environ if environ is None else environ
    d = env.get(parallel.LOCK_DIR_VAR)
    if d:
        return d, "env"
    return parallel.default_lock_dir(env, cwd)


def connectable(path: str, timeout: float = 2.0) -> bool:
    try:
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
            s.settimeout(timeout)
            s.connect(path)
            send_msg(s, {"op": "ping"})
            h, _ = recv_msg(s)
            return h.get("ok") is True
    except OSError:
        return False


# ------------------------------------------------------------------ client
class Client:
    def __init__(self, path: str):
        self.path = path
        self.last: dict = {}

    def _call(self, header: dict, bufs: Sequence = ()) -> Tuple[dict, List[bytearray]]:
        try:
            with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
                s.connect(self.path)
                send_msg(s, header, bufs)
                return recv_msg(s)
        except OSError as e:
            raise ServerUnavailable(str(e)) from e

    def run_chain(self, params, max_total_reads: int, meth_c, tot_c, meth_k, tot_k, seed: int, chain_id: int):
        """One chain in the server: the (BackwardSimulationResults, None, extras)
        of two_group.run (no final weights)."""
        from . import _lib, two_group

        mc, tc = two_group._u16(meth_c), two_group._u16(tot_c)
        mk, tk = two_group._u16(meth_k), two_group._u16(tot_k)
        T = tc.shape[0]
        if mc.shape != tc.shape or mk.shape != tk.shape or tk.shape[0] != T:
            raise ValueError("inconsistent count shapes")
        head = {"op": "chain", "params": bytes(params).hex(), "max_total_reads": int(max_total_reads), "T": int(T),
                "s_c": int(tc.shape[1]), "s_k": int(tk.shape[1]), "seed": int(seed), "chain_id": int(chain_id)}
        h, bufs = self._call(head, (mc, tc, mk, tk))
        self.last = h
        rc = h.get("rc", SERVER_FAULT)
        if rc != 0:
            if rc in _lib.ERROR_NAMES:  # the chain's own failure, as the library reports it in-process
                raise _lib.HygError(int(rc), h.get("error", ""))
            raise ServerUnavailable(h.get("error", "server error"))
        K, B = int(params.n_regimes), int(params.num_samples_backward)
        merged = np.frombuffer(bufs[0], np.int16).reshape(T, B)
        control = np.frombuffer(bufs[1], np.int16).reshape(T, B, 2)
        case = np.frombuffer(bufs[2], np.int16).reshape(T, B, 2)
        split = np.frombuffer(bufs[3], np.float32).reshape(T)
        regime = np.frombuffer(bufs[4], np.float32).reshape(T, 2 * K)
        res = two_group.BackwardSimulationResults(step=np.arange(T), particle={
            "merged_state": merged, "control_state": control, "case_state": case})
        return res, None, {"split_probs": split, "regime_probs": regime, "log_z": float(h["log_z"])}

    def status(self) -> dict:
        return self._call({"op": "status"})[0]

    def stop(self) -> dict:
        return self._call({"op": "stop"})[0]


def task_client(environ=None, cwd: str = None) -> Optional[Client]:
    """The server client of one `hygeia infer` task (a server answers on the
    lock directory's socket and $HYGEIA_SERVER is not "0"), or None: the task
    runs its chain itself."""
    env = os.environ if environ is None else environ
    if env.get(MODE_VAR, "").strip() == "0":
        return None
    path = socket_path(lock_dir(env, cwd)[0])
    return Client(path) if os.path.exists(path) and connectable(path) else None


# ------------------------------------------------------------------ server
class _Request:
    __slots__ = ("header", "bufs", "done", "reply", "t_in")

    def __init__(self, header, bufs):
        self.header, self.bufs = header, bufs
        self.done = threading.Event()
        self.reply: Tuple[dict, list] = ({"rc": SERVER_FAULT, "error": "not run"}, [])
        self.t_in = time.monotonic()

    def key(self):
        h = self.header
        return h["params"], h["s_c"], h["s_k"]


class Engine:
    """Runs a batch of chain requests on one device through the C ABI
    (hyg_tg_run_chains_host: one launch for the batch). Models are cached per
    parameter set and grown when a request needs more reads or sites."""

    def __init__(self, device: int):
        self.device = device
        self.models: Dict[str, Tuple[object, int, int]] = {}

    def start(self) -> None:
        from . import _lib

        self.L = _lib.load(import_torch=False)
        _lib.check(self.L.hyg_set_device(self.device))

    def _model(self, params_hex: str, reads: int, sites: int):
        import ctypes as C

        from . import _lib

        h, r0, s0 = self.models.get(params_hex, (None, -1, -1))
        if h is not None and reads <= r0 and sites <= s0:
            return h
        if h is not None:
            self.L.hyg_tg_model_destroy(h)
            del self.models[params_hex]
        reads, sites = max(reads, r0), max(sites, s0)
        p = _lib.TgParams.from_buffer_copy(bytes.fromhex(params_hex))
        h = C.c_void_p()
        _lib.check(self.L.hyg_tg_model_create(C.byref(p), int(reads), int(sites), C.byref(h)))
        if len(self.models) >= 8:  # the oldest parameter set's model goes
            old = next(iter(self.models))
            self.L.hyg_tg_model_destroy(self.models.pop(old)[0])
        self.models[params_hex] = (h, reads, sites)
        return h

    def run(self, reqs: List[_Request]) -> None:
        import ctypes as C

        from . import _lib

        h0 = reqs[0].header
        p = _lib.TgParams.from_buffer_copy(bytes.fromhex(h0["params"]))
        K, B = int(p.n_regimes), int(p.num_samples_backward)
        s_c, s_k = int(h0["s_c"]), int(h0["s_k"])
        Ts = [int(r.header["T"]) for r in reqs]
        h = self._model(h0["params"], max(int(r.header["max_total_reads"]) for r in reqs), max(Ts))
        R = sum(Ts)
        cat = [np.concatenate([np.frombuffer(r.bufs[i], np.uint16) for r in reqs]) for i in range(4)]
        arr = (_lib.TgChain * len(reqs))()
        off = 0
        for i, r in enumerate(reqs):
            arr[i].site_begin, arr[i].n_sites = off, Ts[i]
            arr[i].seed, arr[i].chain_id, arr[i].out_begin = int(r.header["seed"]), int(r.header["chain_id"]), off
            off += Ts[i]
        merged = np.empty((R, B), np.int16)
        control = np.empty((R, B, 2), np.int16)
        case = np.empty((R, B, 2), np.int16)
        split = np.empty(R, np.float32)
        regime = np.empty((R, 2 * K), np.float32)
        log_z = np.empty(len(reqs), np.float64)
        status = np.empty(len(reqs), np.int32)
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        t0 = time.monotonic()
        rc = self.L.hyg_tg_run_chains_host(h, ptr(cat[0]), ptr(cat[1]), s_c, ptr(cat[2]), ptr(cat[3]), s_k, R, arr,
                                           len(reqs), R, ptr(merged), ptr(control), ptr(case), ptr(split),
                                           ptr(regime), ptr(log_z), None, ptr(status))
        dt = time.monotonic() - t0
        err = self.L.hyg_last_error().decode(errors="replace") if rc else ""
        off = 0
        for i, r in enumerate(reqs):
            T = Ts[i]
            if rc:  # the launch failed (e.g. the batch's memory): each task runs its chain itself
                r.reply = ({"rc": SERVER_FAULT, "error": f"server launch: {err}"}, [])
            elif status[i] != 0:
                r.reply = ({"rc": int(status[i]), "error": "all particle weights became -inf"}, [])
            else:
                sl = slice(off, off + T)
                r.reply = ({"rc": 0, "log_z": float(log_z[i]), "batch": len(reqs), "device": self.device,
                            "wait_s": t0 - r.t_in, "run_s": dt},
                           [merged[sl], control[sl], case[sl], split[sl], regime[sl]])
            off += T


class Server:
    """Accepts chain requests on a UNIX socket; one worker per device takes every
    waiting request with one parameter set when its device comes free and runs
    them as one launch. `engine_factory(device)` makes the per-device engine
    (tests pass a fake one)."""

    def __init__(self, path: str, n_devices: int, engine_factory=Engine, idle: float = IDLE_S,
                 max_batch_sites: int = 16_000_000, gather: float = 0.0):
        self.path, self.idle, self.max_batch_sites = path, float(idle), int(max_batch_sites)
        self.gather = float(gather)  # seconds a free device waits after the oldest request for more to join
        self.pending: List[_Request] = []
        self.cv = threading.Condition()
        self.stopping = False
        self.busy = 0
        self.last_work = time.monotonic()
        self.stats = {"requests": 0, "batches": 0, "chains": 0, "max_batch": 0, "batch_sizes": []}
        self.engines = [engine_factory(d) for d in range(n_devices)]

    # a worker per device
    def _take(self) -> List[_Request]:
        """Under self.cv: the oldest request's parameter set, every waiting
        request with it (up to max_batch_sites sites)."""
        key = self.pending[0].key()
        take, rest, sites = [], [], 0
        for r in self.pending:
            if r.key() == key and (not take or sites + int(r.header["T"]) <= self.max_batch_sites):
                take.append(r)
                sites += int(r.header["T"])
            else:
                rest.append(r)
        self.pending = rest
        return take

    def _worker(self, eng) -> None:
        try:
            eng.start()
        except Exception as e:  # this device is unusable: fail its requests, leave the others
            print(f"[hygeia serve] device {getattr(eng, 'device', '?')}: {e}", file=sys.stderr, flush=True)
            return
        while True:
            with self.cv:
                while not self.pending and not self.stopping:
                    self.cv.wait(0.5)
                if self.stopping and not self.pending:
                    return
                if self.gather > 0:
                    deadline = self.pending[0].t_in + self.gather
                    while not self.stopping and time.monotonic() < deadline:
                        self.cv.wait(max(0.0, deadline - time.monotonic()))
                    if not self.pending:  # another device took them
                        continue
                batch = self._take()
                self.busy += 1
            try:
                eng.run(batch)
            except Exception as e:
                for r in batch:
                    r.reply = ({"rc": SERVER_FAULT, "error": f"server: {e}"}, [])
            with self.cv:
                self.busy -= 1
                self.last_work = time.monotonic()
                self.stats["batches"] += 1
                self.stats["chains"] += len(batch)
                self.stats["max_batch"] = max(self.stats["max_batch"], len(batch))
                self.stats["batch_sizes"] = (self.stats["batch_sizes"] + [len(batch)])[-64:]
            for r in batch:
                r.done.set()

    def _handle(self, conn: socket.socket) -> None:
        with conn:
            try:
                header, bufs = recv_msg(conn)
                op = header.get("op")
                if op == "ping":
                    send_msg(conn, {"ok": True})
                elif op == "status":
                    with self.cv:
                        st = dict(self.stats, pending=len(self.pending), busy=self.busy, pid=os.getpid(),
                                  devices=len(self.engines))
                    send_msg(conn, st)
                elif op == "stop":
                    with self.cv:
                        self.stopping = True
                        self.cv.notify_all()
                    send_msg(conn, {"ok": True})
                elif op == "chain":
                    r = _Request(header, bufs)
                    with self.cv:
                        if self.stopping:
                            send_msg(conn, {"rc": SERVER_FAULT, "error": "server stopping"})
                            return
                        self.stats["requests"] += 1
                        self.pending.append(r)
                        self.cv.notify_all()
                    r.done.wait()
                    send_msg(conn, *r.reply)
                else:
                    send_msg(conn, {"rc": SERVER_FAULT, "error": f"unknown op {op!r}"})
            except (OSError, ValueError, KeyError) as e:
                try:
                    send_msg(conn, {"rc": SERVER_FAULT, "error": f"bad request: {e}"})
                except OSError:
                    pass

    def serve_forever(self) -> None:
        if os.path.exists(self.path):
            os.unlink(self.path)
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(self.path)
        srv.listen(256)
        srv.settimeout(0.5)
        ino = os.stat(self.path).st_ino
        workers = [threading.Thread(target=self._worker, args=(e,), daemon=True) for e in self.engines]
        for w in workers:
            w.start()
        print(f"[hygeia serve] pid {os.getpid()} on {self.path}, {len(self.engines)} device(s)", file=sys.stderr,
              flush=True)
        try:
            while True:
                try:
                    conn, _ = srv.accept()
                    conn.settimeout(None)
                    threading.Thread(target=self._handle, args=(conn,), daemon=True).start()
                except socket.timeout:
                    pass
                with self.cv:
                    idle = (self.idle > 0 and not self.pending and self.busy == 0
                            and time.monotonic() - self.last_work > self.idle)
                    gone = not os.path.exists(self.path) or os.stat(self.path).st_ino != ino
                    if self.stopping or idle or gone or not any(w.is_alive() for w in workers):
                        self.stopping = True
                        self.cv.notify_all()
                        break
        finally:
            for w in workers:
                w.join(timeout=600)
            with self.cv:  # requests no worker took (every device failed): their tasks run them
                left, self.pending = self.pending, []
            for r in left:
                r.reply = ({"rc": SERVER_FAULT, "error": "server: no usable device"}, [])
                r.done.set()
            srv.close()
            try:
                if os.stat(self.path).st_ino == ino:
                    os.unlink(self.path)
            except OSError:
                pass
            print(f"[hygeia serve] exit: {json.dumps({k: v for k, v in self.stats.items() if k != 'batch_sizes'})}",
                  file=sys.stderr, flush=True)


def main(argv: Sequence[str] = None) -> int:
    """`hygeia serve [--socket PATH] [--idle S] [--stop | --status]`."""
    import argparse

    ap = argparse.ArgumentParser(prog="hygeia serve")
    ap.add_argument("--socket", default=None, help="default: the device lock directory's server socket")
    ap.add_argument("--idle", type=float, default=IDLE_S, help="exit after this many seconds without work (0: never)")
    ap.add_argument("--gather", type=float, default=0.0,
                    help="seconds a free GPU waits after the oldest waiting chain for others to join its launch")
    ap.add_argument("--stop", action="store_true", help="stop the running server (after its current launches)")
    ap.add_argument("--status", action="store_true")
    a = ap.parse_args(argv)
    path = a.socket or socket_path(lock_dir()[0])
    if a.stop or a.status:
        c = Client(path)
        try:
            print(json.dumps(c.stop() if a.stop else c.status()))
        except ServerUnavailable:
            print(json.dumps({"running": False, "socket": path}))
            return 1 if a.status else 0
        if a.stop:
            t0 = time.monotonic()
            while os.path.exists(path) and time.monotonic() - t0 < 600:
                time.sleep(0.1)
        return 0
    from . import _lib

    L = _lib.load(import_torch=False)
    n = int(L.hyg_device_count())
    if n < 1:
        print("hygeia serve: no HIP device", file=sys.stderr)
        return 1
    Server(path, n, idle=a.idle, gather=a.gather).serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())

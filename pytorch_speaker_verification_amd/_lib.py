"""Loader for the in-tree gfx950 HIP library (libsv_ge2e.so) behind include/sv_ge2e.h.

There is no fallback: if the library is missing or fails to load, every op raises.
The library binds to the HIP runtime torch already loaded (same soname,
libamdhip64.so.7), so torch must be imported first -- this module does that.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsv_ge2e.so")
# the fault-injection test build (Makefile `faultinj`): the same library plus sv_test_set_fault;
# only tests load it, through use_library() before the first call
FAULT_LIB_PATH = os.path.join(_HERE, "libsv_ge2e_faultinj.so")
ABI_VERSION = 11
SV_DTYPE_F32, SV_DTYPE_BF16 = 0, 1  # include/sv_ge2e.h

# schedule flags of the bf16 stack (include/sv_ge2e.h SV_SCHED_*), by name
SCHEDULES = {"auto": 0, "per_layer": 1, "per_step": 2, "persist": 5}  # persist: per-layer persistent, any H
SV_SCHED_NO_EVENTS = 8  # the stack backward records no per-layer completion events (nothing waits on them)
SV_SCHED_WT_READY = 16  # the bf16 backward workspace already holds sv_lstm_weights_bf16's transposes
SV_SCHED_CNT_READY = 32  # the bf16 backward's counter channels are as the last stack forward zeroed them


def schedule_flags(schedule):
    """'auto' | 'per_layer' | 'per_step' | 'persist' (or an int of SV_SCHED_* flags) -> int."""
    if schedule is None:
        return 0
    if isinstance(schedule, int):
        if schedule & ~7:
            raise ValueError(f"unknown schedule flags {schedule:#x}")
        return schedule
    try:
        return SCHEDULES[schedule]
    except KeyError:
        raise ValueError(f"unknown schedule {schedule!r} (expected one of {sorted(SCHEDULES)})") from None

_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_long = ctypes.c_long
_c_float = ctypes.c_float
_c_size_t = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/sv_ge2e.h
_P = _c_void_p
SIGNATURES = {
    "sv_abi_version": (_c_int, []),
    "sv_gemm_f32_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_gemm_f32": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _c_long, _P, _c_long, _P, _P,
                             _c_float, _P, _c_int, _P]),
    "sv_colsum_workspace": (_c_size_t, [_c_int, _c_int]),
    "sv_colsum": (_c_int, [_P, _c_int, _c_int, _P, _P, _P]),
    "sv_frames_to_time_major": (_c_int, [_P, _P, _c_int, _c_int, _c_int, _P]),
    "sv_transpose": (_c_int, [_P, _c_long, _c_int, _c_int, _P, _c_long, _P]),
    "sv_lstm_layer_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_lstm_step_fwd": (_c_int, [_P, _P, _P, _P, _P, _P, _c_int, _c_int, _P]),
    "sv_lstm_step_bwd": (_c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _c_int, _c_int, _P]),
    "sv_lstm_stack_fwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _c_int, _P, _P, _P, _c_int, _c_int, _P, _P]),
    "sv_lstm_f32_persist_ok": (_c_int, [_c_int, _c_int, _c_int]),
    "sv_lstm_stack_bwd_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_stack_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int] + [_P] * 16 + [_c_int, _P, _P, _P, _c_int,
                                                                                          _P, _P, _c_int, _P]),
    "sv_lstm_layer_bwd_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_layer_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _P, _P, _P, _P, _P, _c_int, _P,
                                   _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_proj_norm_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_proj_norm_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_proj_norm_bwd": (_c_int, [_P, _P, _P, _P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_workspace_size": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_ge2e_speaker_sums": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P]),
    "sv_ge2e_fwd_rows": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd_rows": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd_finalize": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd": (_c_int, [_c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_train_ok": (_c_int, [_c_int, _c_int, _c_int]),
    "sv_ge2e_train": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_shard_prep": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P]),
    "sv_ge2e_shard_rows": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_shard_finalize": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P]),
    "sv_ge2e_centroids": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P]),
    "sv_ge2e_cossim_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_ge2e_cossim": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _c_int, _P, _P, _P]),
    "sv_ge2e_calc_loss": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P]),
    "sv_ge2e_centroids_bwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P]),
    "sv_ge2e_cossim_bwd_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_ge2e_cossim_bwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _c_int, _P, _P, _P, _P, _P]),
    "sv_ge2e_calc_loss_bwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P]),
    "sv_gemm_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_gemm_bf16": (_c_int, [_c_int, _c_int, _c_int, _P, _c_long, _P, _c_long, _P, _c_long, _P, _P, _c_float, _P,
                              _P]),
    "sv_gemm_bf16_bf": (_c_int, [_c_int, _c_int, _c_int, _P, _c_long, _P, _c_long, _P, _c_long, _P, _P, _P]),
    "sv_cast_bf16": (_c_int, [_P, _P, _c_long, _P]),
    "sv_cast_bf16_batch": (_c_int, [_c_int, _P, _P, _P, _P]),
    "sv_transpose_cast_bf16": (_c_int, [_P, _c_long, _c_int, _c_int, _P, _c_long, _P]),
    "sv_frames_to_bf16": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _c_int, _P]),
    "sv_lstm_weights_bf16": (_c_int, [_c_int] * 5 + [_P] * 6),
    "sv_lstm_prep_bf16": (_c_int, [_c_int] * 5 + [_P] * 3 + [_c_int] + [_P] * 6),
    "sv_lstm_layer_fwd_bf16": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_lstm_stack_fwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _P, _c_int, _P, _P, _P, _P, _P, _c_int]),
    "sv_lstm_layer_bwd_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_layer_bwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _P, _P, _P, _P, _P, _c_int,
                                        _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_eer_counts": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _c_int, _P, _P, _P]),
    "sv_lstm_stack_bwd_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_stack_bwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int] + [_P] * 16 + [_c_int, _P, _P, _P, _P,
                                                                                               _P, _c_int]),
    # dtype-enum form of the stack entry points (SV_DTYPE_F32 / SV_DTYPE_BF16)
    "sv_lstm_fwd": (_c_int, [_c_int] * 6 + [_P] * 10 + [_c_int, _P, _P, _P, _c_int, _c_int, _P, _P]),
    "sv_lstm_bwd_workspace": (_c_size_t, [_c_int] * 6),
    "sv_lstm_bwd": (_c_int, [_c_int] * 6 + [_P] * 16 + [_c_int, _P, _P, _P, _c_int, _P, _P, _c_int, _P]),
    "sv_sync_size": (_c_size_t, []),
    "sv_persist_fwd_ok": (_c_int, [_c_int, _c_int]),
    "sv_persist_bwd_ok": (_c_int, [_c_int, _c_int]),
    "sv_wave_ok": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_persist_bwd_scratch": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_status_poison": (_c_int, [_P, _P, _c_int, _P]),
    "sv_status_report": (_c_int, [_P, _P, _c_int, _P, ctypes.c_uint, _P]),
    "sv_host_device_ptr": (_c_int, [_P, _P]),
    "sv_status_to_flag": (_c_int, [_P, _P, _P]),
    "sv_status_merge": (_c_int, [_P, _P, _P]),
    "sv_dvector_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_dvector_embed_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _c_int, _P,
                                       _P, _P]),
    "sv_clip_sgd_workspace": (_c_size_t, []),
    "sv_clip_sgd_step": (_c_int, [_P, _P, _c_long, _c_float, _c_float, _c_int, _P, _P, _P, _P]),
    "sv_clip_sgd_step2": (_c_int, [_P, _P, _c_long, _c_float, _P, _P, _c_long, _c_float, _c_float, _c_int, _P, _P, _P,
                                   _P]),
    "sv_clip_sgd_step2_report": (_c_int, [_P, _P, _c_long, _c_float, _P, _P, _c_long, _c_float, _c_float, _c_int, _P,
                                          _P, _P, _P, _c_int, _P, ctypes.c_uint, _P]),
}

ERRORS = {-1: "invalid argument (SV_EARG)", -2: "misaligned pointer/leading dim (SV_EALIGN)",
          -3: "unsupported shape (SV_ESHAPE)"}

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def use_library(path):
    """Load ``path`` instead of the shipped library (tests: the fault-injection build).  Must run
    before the first call into the library in this process."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise NativeLibraryError(f"{LIB_PATH} is already loaded")
    LIB_PATH = path


def lib():
    """The loaded library (loaded once).  Raises NativeLibraryError if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `make` (or __graft_entry__.build()); "
                "there is no non-native fallback")
        try:
            h = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        if h.sv_abi_version() != ABI_VERSION:
            raise NativeLibraryError(f"{LIB_PATH} has ABI {h.sv_abi_version()}, expected {ABI_VERSION}: rebuild it")
        if hasattr(h, "sv_test_set_fault"):
            h.sv_test_set_fault.restype = _c_int
            h.sv_test_set_fault.argtypes = [_c_int]
        _lib = h
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = ERRORS.get(rc, f"HIP error {rc}")
        raise RuntimeError(f"{name} failed: {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(t):
    """hipStream_t of the current stream on the tensor's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


class PersistentRecurrenceError(RuntimeError):
    """A persistent recurrence's hand-off wait timed out (its grid was not co-resident: another
    kernel or process held CUs it needed).  Outputs since then are invalid; the trainer's
    clip + SGD step skipped the update (include/sv_ge2e.h, sync block)."""


class PersistStatus:
    """A caller-owned sync block for the persistent recurrences (sv_sync_size bytes, zeroed once)
    plus a non-blocking check of its sticky status word: ``arm()`` after enqueueing work that
    uses the block issues an async device->pinned copy of the word behind it; ``report(x)``
    (the training step's end) instead poisons x on a timeout and has one kernel store the word
    into a ring of pinned host slots (sv_status_report: no copy, no event); ``poll()`` raises
    PersistentRecurrenceError for any completed check that saw a nonzero status (``wait=True``
    first waits for all of them)."""

    RING = 64

    def __init__(self, device):
        words = (int(lib().sv_sync_size()) + 3) // 4
        self.block = torch.zeros(words, dtype=torch.int32, device=device)
        self._pending = []
        self._ring = None  # pinned host slots of sv_status_report, set up on first use
        self._seq = 0
        # the bf16 stack forward zeroed the block's backward counter channels and no backward has
        # run on it since (ops.py: the next bf16 backward passes SV_SCHED_CNT_READY)
        self.bwd_counters_clean = False

    def ptr(self):
        return self.block.data_ptr()

    def report(self, x):
        """x (fp32, contiguous, on the block's device) := NaN if the status is set, and the status
        reported into the next host slot, both stream-ordered on x's stream (sv_status_report)."""
        slot, seq = self.next_slot()
        call("sv_status_report", self.ptr(), ptr(x), x.numel(), slot, seq, stream_of(x))

    def next_slot(self):
        """(device address, sequence number) of the next host report slot, registered as a pending
        check: the caller's launch (sv_status_report, or the trainer's sv_clip_sgd_step2_report)
        must store (seq << 32) | status there."""
        if self._ring is None:
            ring = torch.zeros(self.RING, dtype=torch.int64, pin_memory=True)
            dev = ctypes.c_void_p()
            rc = lib().sv_host_device_ptr(ctypes.c_void_p(ring.data_ptr()), ctypes.byref(dev))
            if rc != 0 or not dev.value:
                raise NativeLibraryError(f"sv_host_device_ptr failed ({rc}): pinned host memory is not mapped")
            self._ring, self._ring_dev = ring, dev.value
        if sum(1 for p in self._pending if p[0] == "slot") >= self.RING - 1:
            self.poll(wait=True)  # every slot in use: the host is a whole ring ahead of the device
        self._seq = self._seq % 0xFFFFFFFF + 1  # (never 0: a fresh slot reads 0)
        k = self._seq % self.RING
        self._pending.append(("slot", k, self._seq))
        return self._ring_dev + 8 * k, self._seq

    def arm(self):
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(self.block[:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.block.device))
        self._pending.append(("copy", ev, host))

    def poll(self, wait=False):
        keep = []
        bad = 0
        if wait and any(p[0] == "slot" for p in self._pending):
            torch.cuda.synchronize(self.block.device)
        for p in self._pending:
            if p[0] == "slot":
                v = int(self._ring[p[1]])
                if (v >> 32) == p[2]:
                    bad |= v & 0xFFFFFFFF
                else:
                    keep.append(p)
                continue
            _, ev, host = p
            if wait:
                ev.synchronize()
            if ev.query():
                bad |= int(host[0])
            else:
                keep.append(p)
        self._pending = keep
        if bad:
            which = " and ".join(n for b, n in ((1, "forward"), (2, "backward")) if bad & b)
            raise PersistentRecurrenceError(
                f"a persistent {which} recurrence timed out waiting for a hand-off (status {bad}): its grid was not "
                "co-resident; the step's outputs are invalid and its parameter update was skipped")

    def clear(self):
        """Forget pending checks and zero the status word (stream-ordered)."""
        self._pending = []
        self.block[:1].zero_()


def compute_device(t):
    """The GPU a tensor's op runs on: its own device if it is on one, else (a CPU tensor, as in
    the reference's CPU-resident evaluation, train_speech_embedder.py:100-102,120-121) the
    current HIP device -- the data makes a round trip there and back; there is no CPU path."""
    if t.is_cuda:
        return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("pytorch_speaker_verification_amd ops run on the GPU only (HIP kernels, no CPU "
                           f"fallback) and no GPU is visible (got a {t.device} tensor)")
    return torch.device("cuda", torch.cuda.current_device())


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("pytorch_speaker_verification_amd ops run on the GPU only "
                               f"(got a {t.device} tensor); move the module/tensors with .to('cuda')")
        if t.dtype != torch.float32:
            raise RuntimeError(f"expected float32 tensors, got {t.dtype}")
        if not t.is_contiguous():
            raise RuntimeError("expected contiguous tensors")

"""Device-scope HIP events (ctypes over the HIP runtime torch already loaded).

torch.cuda.Event records with a system-scope release: the command processor writes back and
invalidates the caches at the record, ~6 us of idle GPU between the kernels either side
(tools/event_cost.py).  Ordering two streams of the same device needs only a device-scope release,
hipEventDisableSystemFence -- used for every stream-to-stream dependency of the step.  The host never
waits on these (the loss copy to pinned memory keeps a torch event)."""
import ctypes

import torch

_HIP = None
DISABLE_TIMING = 0x2
DISABLE_SYSTEM_FENCE = 0x20000000


def _hip():
    global _HIP
    if _HIP is None:
        torch.cuda.init()
        h = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same SONAME)
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        h.hipEventDestroy.argtypes = [ctypes.c_void_p]
        h.hipEventQuery.argtypes = [ctypes.c_void_p]
        for f in (h.hipEventCreateWithFlags, h.hipEventRecord, h.hipStreamWaitEvent, h.hipEventDestroy,
                  h.hipEventQuery):
            f.restype = ctypes.c_int
        _HIP = h
    return _HIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def _sp(stream):
    return ctypes.c_void_p((stream if stream is not None else torch.cuda.current_stream()).cuda_stream)


class DeviceEvent:
    """Orders one stream after work recorded on another, device scope only."""

    def __init__(self):
        h = _hip()
        self._ev = ctypes.c_void_p()
        _check(h.hipEventCreateWithFlags(ctypes.byref(self._ev), DISABLE_TIMING | DISABLE_SYSTEM_FENCE),
               "hipEventCreateWithFlags")

    def record(self, stream=None):
        _check(_hip().hipEventRecord(self._ev, _sp(stream)), "hipEventRecord")
        return self

    def wait(self, stream=None):
        """Make `stream` (default: torch's current) wait for the recorded work."""
        _check(_hip().hipStreamWaitEvent(_sp(stream), self._ev, 0), "hipStreamWaitEvent")

    def __del__(self):
        if _HIP is not None and self._ev:
            _HIP.hipEventDestroy(self._ev)


def wait_stream(waiter, other):
    """waiter waits for everything queued so far on other (torch's Stream.wait_stream, device scope)."""
    DeviceEvent().record(other).wait(waiter)


HOST_MALLOC_MAPPED = 0x2
HOST_MALLOC_COHERENT = 0x40000000


class MappedHostBuffer:
    """Small pinned host buffer the GPU writes directly (hipHostMallocMapped | Coherent): the
    step's loss scalars land here from the finalize kernel, which then stores a sequence word the
    host polls -- no device->host copy and no event on the compute stream."""

    def __init__(self, nwords=16):
        import numpy as np

        h = _hip()
        h.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        h.hipHostMalloc.restype = ctypes.c_int
        h.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
        h.hipHostGetDevicePointer.restype = ctypes.c_int
        h.hipHostFree.argtypes = [ctypes.c_void_p]
        h.hipHostFree.restype = ctypes.c_int
        self._p = ctypes.c_void_p()
        _check(h.hipHostMalloc(ctypes.byref(self._p), 4 * nwords, HOST_MALLOC_MAPPED | HOST_MALLOC_COHERENT),
               "hipHostMalloc")
        self._d = ctypes.c_void_p()
        _check(h.hipHostGetDevicePointer(ctypes.byref(self._d), self._p, 0), "hipHostGetDevicePointer")
        raw = (ctypes.c_uint32 * nwords).from_address(self._p.value)
        self.u32 = np.frombuffer(raw, dtype=np.uint32)
        self.f32 = np.frombuffer(raw, dtype=np.float32)
        self.u32[:] = 0

    @property
    def device_ptr(self):
        return self._d

    def wait(self, index, value, timeout=60.0):
        """Spin until word `index` equals `value` (the GPU's release store); on timeout, surface any
        device error through torch.cuda.synchronize() before giving up."""
        import time

        w = self.u32
        if w[index] == value:
            return
        t0 = time.perf_counter()
        while w[index] != value:
            if time.perf_counter() - t0 > timeout:
                torch.cuda.synchronize()
                if w[index] == value:
                    return
                raise RuntimeError(f"mapped host word {index} never reached {value} (got {int(w[index])})")

    def __del__(self):
        if _HIP is not None and self._p:
            _HIP.hipHostFree(self._p)

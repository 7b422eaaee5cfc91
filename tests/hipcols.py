"""Device-resident history columns for GPU tests: hipMalloc + hipMemcpy
through the HIP runtime libjh.so already loaded (torch would load a second
runtime into the process)."""
import numpy as np


class DevCols:
    """The columns copied to device memory (hipMalloc through the HIP runtime
    libjh.so already loaded -- no second runtime from torch in this process),
    each starting `shift` int64s into its allocation (shift 1: 8-byte aligned
    only)."""

    def __init__(self, cols, shift):
        import ctypes as C
        from jepsen_amd import _native
        _native.lib()
        path = next((ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln), "libamdhip64.so")
        self._hip = hip = C.CDLL(path)
        hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        hip.hipFree.argtypes = [C.c_void_p]
        self._bufs = []
        self.n, self.n_keys = int(cols.n), int(cols.n_keys)

        def put(a):
            a = np.ascontiguousarray(a, dtype=np.int64)
            p = C.c_void_p()
            rc = hip.hipMalloc(C.byref(p), 8 * (len(a) + shift + 1))
            if rc != 0:
                hip.hipGetErrorString.restype = C.c_char_p
                raise AssertionError(f"hipMalloc({8 * (len(a) + shift + 1)} B) -> {rc} "
                                     f"{hip.hipGetErrorString(rc).decode()}")
            self._bufs.append(p)
            dst = p.value + 8 * shift
            assert hip.hipMemcpy(dst, a.ctypes.data, 8 * len(a), 1) == 0       # hipMemcpyHostToDevice
            return dst
        for k in ("process", "type", "f", "key", "value", "value2"):
            setattr(self, k, put(getattr(cols, k)))
        self.aux, self.n_aux = put(cols.aux), len(cols.aux)

    def __del__(self):
        for p in getattr(self, "_bufs", []):
            self._hip.hipFree(p)

"""Host arrays and kernel-parameter groups.

MI355X-native counterparts of the reference's array layer:

* :class:`FastArr` and the typed ``Cl*Array`` classes — pinned, page-aligned
  host arrays (``hipHostMalloc`` portable+mapped, visible to all GPUs), the
  equivalent of ``FastArr<T>``/``ClFloatArray``… (CSpaceArrays.cs:234-1517).
* :class:`ClArray` — wraps a numpy array, a torch CPU tensor or a
  :class:`FastArr` and carries the per-array transfer flags that decide what
  ``compute()`` moves (ClArray.cs:717-1907; flag rules :1742-1888).
* :class:`ClParameterGroup` — an ordered list of arrays that become the
  kernel's parameters (``nextParam`` chaining, ClArray.cs:155-660).

Flag semantics: ``partial_read`` uploads only a device's slice
``[ref·e, (ref+r)·e)`` and wins over ``read`` (whole array to every device);
``write`` downloads the device's slice; ``write`` + ``write_all`` makes device
``(array index mod D)`` download the whole array; ``read_only``/``write_only``
clear the conflicting flags; ``zero_copy`` lets kernels access the pinned host
memory directly (no copies).
"""
from __future__ import annotations

import ctypes
import itertools
import threading
import weakref
from typing import Iterable, Optional, Sequence, Union

import numpy as np

from ._native import cek

# --------------------------------------------------------------------------- dtypes

BFLOAT16 = "bfloat16"

_DTYPES = {
    "float32": np.float32, "float": np.float32, "f32": np.float32,
    "float64": np.float64, "double": np.float64, "f64": np.float64,
    "int32": np.int32, "int": np.int32, "uint32": np.uint32, "uint": np.uint32,
    "int64": np.int64, "long": np.int64, "uint64": np.uint64,
    "uint8": np.uint8, "byte": np.uint8, "int8": np.int8,
    "int16": np.int16, "uint16": np.uint16, "char": np.uint16,  # C# char = 16 bit
    "float16": np.float16, "half": np.float16,
}


def _resolve_dtype(dtype) -> tuple[np.dtype, bool]:
    """Returns (numpy storage dtype, is_bf16)."""
    if dtype is None:
        return np.dtype(np.float32), False
    if isinstance(dtype, str):
        key = dtype.lower()
        if key in ("bfloat16", "bf16"):
            return np.dtype(np.uint16), True
        if key in _DTYPES:
            return np.dtype(_DTYPES[key]), False
    try:
        import torch

        if isinstance(dtype, torch.dtype):
            if dtype == torch.bfloat16:
                return np.dtype(np.uint16), True
            return np.dtype(torch.empty(0, dtype=dtype).numpy().dtype), False
    except Exception:  # pragma: no cover
        pass
    return np.dtype(dtype), False


_uid_counter = itertools.count(1)
_live_cores: "weakref.WeakSet" = weakref.WeakSet()
# re-entrant: a garbage collection inside the locked region can run a
# ClArray.__del__ that releases its uid on the same thread
_live_lock = threading.RLock()


def _register_cores(c) -> None:
    with _live_lock:
        _live_cores.add(c)


def _release_uid(uid: int) -> None:
    with _live_lock:
        cores = list(_live_cores)
    for c in cores:
        try:
            c._release_array(uid)
        except Exception:
            pass


# --------------------------------------------------------------------------- FastArr


class FastArr:
    """Pinned, aligned native host array (reference ``FastArr<T>``).

    Allocated with ``hipHostMalloc(portable | mapped)`` when a GPU is present
    (falls back to ``posix_memalign`` on CPU-only hosts).  ``array`` is a numpy
    view of the memory; kernels on any GPU can also read it in place
    (zero-copy).
    """

    def __init__(self, n: int, dtype=np.float32, alignment: int = 4096):
        np_dtype, self.is_bf16 = _resolve_dtype(dtype)
        if n <= 0:
            raise ValueError("FastArr length must be positive")
        self._n = int(n)
        self.alignment = int(alignment)
        nbytes = self._n * np_dtype.itemsize
        self._ptr = cek.host_alloc(nbytes, max(64, self.alignment))
        buf = (ctypes.c_uint8 * nbytes).from_address(self._ptr)
        self._array = np.frombuffer(buf, dtype=np_dtype, count=self._n)
        self._array[...] = 0
        self._disposed = False

    # reference API ------------------------------------------------------------
    @property
    def array(self) -> np.ndarray:
        self._check()
        return self._array

    @property
    def Length(self) -> int:  # noqa: N802
        return self._n

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        return self.array[i]

    def __setitem__(self, i, v):
        self.array[i] = v

    def ha(self) -> int:
        """Aligned head address (reference ``ha()``)."""
        return self._ptr

    def ToArray(self) -> np.ndarray:  # noqa: N802
        return self.array.copy()

    to_array = ToArray

    def CopyTo(self, dst, offset: int = 0) -> None:  # noqa: N802
        src = self.array
        dst_arr = dst.array if hasattr(dst, "array") else dst
        dst_arr[offset:offset + len(src)] = src

    copy_to = CopyTo

    def CopyFrom(self, src, offset: int = 0) -> None:  # noqa: N802
        s = src.array if hasattr(src, "array") else np.asarray(src)
        self.array[offset:offset + len(s)] = s

    copy_from = CopyFrom

    # native-to-native copies of elements [index, N) between equal-length
    # arrays (FastArr.CopyTo_ / CopyFrom_, CSpaceArrays.cs:710-740)
    def CopyTo_(self, dst: "FastArr", index: int = 0) -> None:  # noqa: N802
        if len(dst) != len(self):
            raise ValueError("CopyTo_ needs arrays of equal length")
        dst.array[index:] = self.array[index:]

    def CopyFrom_(self, src: "FastArr", index: int = 0) -> None:  # noqa: N802
        if len(src) != len(self):
            raise ValueError("CopyFrom_ needs arrays of equal length")
        self.array[index:] = src.array[index:]

    @property
    def pinned(self) -> bool:
        return bool(cek.host_is_pinned(self._ptr))

    def _check(self) -> None:
        if self._disposed:
            raise RuntimeError("FastArr used after dispose()")

    def dispose(self) -> None:
        if not self._disposed:
            self._disposed = True
            self._array = None
            cek.host_free(self._ptr)

    def __del__(self):
        try:
            self.dispose()
        except Exception:
            pass


def _typed_fastarr(name: str, dtype):
    cls = type(name, (FastArr,), {
        "__init__": lambda self, n, alignment=4096: FastArr.__init__(self, n, dtype, alignment),
        "__doc__": f"Pinned aligned host array of {dtype} (reference {name}).",
    })
    return cls


ClFloatArray = _typed_fastarr("ClFloatArray", np.float32)
ClDoubleArray = _typed_fastarr("ClDoubleArray", np.float64)
ClIntArray = _typed_fastarr("ClIntArray", np.int32)
ClUIntArray = _typed_fastarr("ClUIntArray", np.uint32)
ClLongArray = _typed_fastarr("ClLongArray", np.int64)
ClByteArray = _typed_fastarr("ClByteArray", np.uint8)
ClCharArray = _typed_fastarr("ClCharArray", np.uint16)
ClBf16Array = _typed_fastarr("ClBf16Array", BFLOAT16)


# --------------------------------------------------------------------------- ClArray

ArrayLike = Union[np.ndarray, FastArr, "ClArray", Sequence]


class ClArray:
    """A kernel-parameter array with transfer flags (reference ``ClArray<T>``).

    Wrapped host memory of at least ``ClArray.auto_pin_min_bytes`` (64 KiB;
    0 disables) is registered with HIP (``hipHostRegister``) on its first
    compute, so its copies are DMA from pinned pages like a FastArr's.

    ``ClArray(n, dtype)`` allocates pinned native memory (like
    ``new ClArray<float>(n)``); ``ClArray(ndarray)`` / ``ClArray(tensor)``
    wraps existing host memory without copying (like the implicit
    ``float[] → ClArray<float>`` conversion, ClArray.cs:1014).
    """

    auto_pin_min_bytes = 64 * 1024

    def __init__(self, data: Union[int, ArrayLike, None] = None, dtype=None, alignment: int = 4096,
                 fast: Optional[bool] = None):
        self._uid = next(_uid_counter)
        self.alignment_bytes = int(alignment)
        self._fast: Optional[FastArr] = None
        self._np: Optional[np.ndarray] = None
        self._torch_ref = None
        self.is_bf16 = False
        if data is None:
            self._np = None
        elif isinstance(data, (int, np.integer)):
            n = int(data)
            if fast is False:
                np_dtype, self.is_bf16 = _resolve_dtype(dtype)
                self._np = np.zeros(n, np_dtype)
            else:
                self._fast = FastArr(n, dtype or np.float32, alignment)
                self.is_bf16 = self._fast.is_bf16
        elif isinstance(data, FastArr):
            self._fast = data
            self.is_bf16 = data.is_bf16
        elif isinstance(data, ClArray):
            self._fast, self._np, self.is_bf16 = data._fast, data._np, data.is_bf16
        else:
            self._wrap_host(data, dtype)
        # reference defaults (ClArray.cs:838-845)
        self._read = True
        self._partial = False
        self._write = True
        self._write_all = False
        self._ro = False
        self._wo = False
        self.zero_copy = False
        self.elements_per_work_item = 1
        # extension: >0 means N elements per work-GROUP (per-group outputs such
        # as reduction partials); the slice of a device is then
        # [ref/L·N, (ref+r)/L·N)
        self.elements_per_group = 0
        # extension: keep-resident gather — after the
        # kernels every device's slice of this array is copied into every
        # other device's replica (GPU↔GPU over xGMI, RCCL across ranks)
        self.gather_resident = False
        # explicit per-blob slices for a compute with explicit pipeline blobs
        # (compute(..., blob_bounds=...)): ((first element, count) per blob),
        # e.g. row panel k of a GEMM operand for shell k; None: the slice
        # proportional to each blob's work items
        self.blob_slices = None
        # per cruncher (id): the split of the last compute this array took
        # part in without the read-only hint — (compute id, elements per work
        # item, elements per group, local range).  A device-resident array's
        # replicas each hold the slice of that split (checkpoint.save).
        self._split_log = {}
        self._registered = False
        self._disposed = False

    def _wrap_host(self, data, dtype) -> None:
        try:
            import torch

            if isinstance(data, torch.Tensor):
                if data.device.type != "cpu":
                    raise ValueError("ClArray wraps host memory; got a tensor on " + str(data.device))
                t = data.contiguous().view(-1)
                self._torch_ref = t
                if t.dtype == torch.bfloat16:
                    self.is_bf16 = True
                    self._np = t.view(torch.int16).numpy().view(np.uint16)
                else:
                    self._np = t.numpy()
                return
        except ImportError:  # pragma: no cover
            pass
        arr = np.asarray(data)
        if dtype is not None:
            np_dtype, self.is_bf16 = _resolve_dtype(dtype)
            if arr.dtype != np_dtype:
                arr = arr.astype(np_dtype)
        if not arr.flags.c_contiguous:
            arr = np.ascontiguousarray(arr)
        self._np = arr.reshape(-1)

    # ------------------------------------------------------------------ storage
    @property
    def array(self) -> np.ndarray:
        """Flat numpy view of the host storage."""
        if self._fast is not None:
            return self._fast.array
        if self._np is None:
            raise ValueError("ClArray has no storage (N not set)")
        return self._np

    @property
    def fast_arr(self) -> bool:
        return self._fast is not None

    @fast_arr.setter
    def fast_arr(self, on: bool) -> None:
        """Switch storage between a native FastArr and a plain numpy array,
        keeping the contents (reference ``fastArr`` setter, ClArray.cs:889)."""
        if on and self._fast is None:
            old = self.array
            f = FastArr(len(old), BFLOAT16 if self.is_bf16 else old.dtype, self.alignment_bytes)
            f.array[:] = old
            self._release_device()
            self._fast, self._np, self._torch_ref = f, None, None
            self._uid = next(_uid_counter)
        elif not on and self._fast is not None:
            self._np = self._fast.array.copy()
            self._release_device()
            self._fast.dispose()
            self._fast = None
            self._uid = next(_uid_counter)

    @property
    def N(self) -> int:  # noqa: N802
        return 0 if (self._fast is None and self._np is None) else len(self.array)

    @N.setter
    def N(self, n: int) -> None:  # noqa: N802
        """Reallocate with the new length (contents not kept; the reference
        allocates with the old N here, a bug not reproduced: ClArray.cs:763)."""
        np_dtype = self.array.dtype if self.N else np.dtype(np.float32)
        self._release_device()
        if self._fast is not None:
            self._fast.dispose()
            self._fast = FastArr(n, BFLOAT16 if self.is_bf16 else np_dtype, self.alignment_bytes)
        else:
            self._np = np.zeros(n, np_dtype)
        self._uid = next(_uid_counter)

    def __len__(self) -> int:
        return self.N

    Length = property(lambda self: self.N)
    Count = Length
    arrayLength = Length

    @property
    def dtype(self):
        return BFLOAT16 if self.is_bf16 else self.array.dtype

    @property
    def itemsize(self) -> int:
        return self.array.itemsize

    @property
    def nbytes(self) -> int:
        return self.array.nbytes

    def host_pointer(self) -> int:
        return self.array.ctypes.data

    def __getitem__(self, i):
        return self.array[i]

    def __setitem__(self, i, v):
        self.array[i] = v

    # The reference's IList<T> members (ClArray.cs:1105-1353) are all
    # NotImplementedException stubs there.  Here the read-only queries work
    # on the host array.  The size-changing ones stay refused: a ClArray has a
    # fixed length that its device buffers mirror.
    def __iter__(self):
        return iter(self.array)

    def __contains__(self, item) -> bool:
        return bool(np.any(self.array == item))

    def contains(self, item) -> bool:
        return item in self

    def index_of(self, item) -> int:
        """First index of ``item`` in the host array, -1 if absent (IList.IndexOf)."""
        hits = np.flatnonzero(self.array == item)
        return int(hits[0]) if len(hits) else -1

    is_read_only = property(lambda self: False)

    def _fixed_size(self, *args, **kwargs):
        raise NotImplementedError("a ClArray has a fixed length (its device buffers mirror it); "
                                  "resize by creating a new ClArray")

    Contains, IndexOf, IsReadOnly, GetEnumerator = contains, index_of, is_read_only, __iter__
    Add = Insert = Remove = RemoveAt = Clear = _fixed_size

    def ToArray(self) -> np.ndarray:  # noqa: N802
        return self.array.copy()

    to_array = ToArray

    def CopyTo(self, dst, offset: int = 0) -> None:  # noqa: N802
        dst_arr = dst.array if hasattr(dst, "array") else dst
        dst_arr[offset:offset + self.N] = self.array

    copy_to = CopyTo

    def CopyFrom(self, src, offset: int = 0) -> None:  # noqa: N802
        s = src.array if hasattr(src, "array") else np.asarray(src).reshape(-1)
        self.array[offset:offset + len(s)] = s

    copy_from = CopyFrom

    def as_torch(self):
        """Zero-copy torch CPU tensor view (bf16 arrays come back as bfloat16)."""
        import torch

        t = torch.from_numpy(self.array)
        if self.is_bf16:
            t = t.view(torch.bfloat16)
        return t

    @staticmethod
    def wrap_array_of_structs(structs: np.ndarray) -> "ClArray":
        """View a structured/record numpy array as a byte array (reference
        ``wrapArrayOfStructs``, ClArray.cs:1058-1074)."""
        s = np.ascontiguousarray(structs)
        return ClArray(s.view(np.uint8).reshape(-1))

    wrapArrayOfStructs = wrap_array_of_structs

    # -------------------------------------------------------------------- flags
    @property
    def read(self) -> bool:
        return self._read

    @read.setter
    def read(self, v: bool) -> None:
        if not self._wo:
            self._read = bool(v)

    @property
    def partial_read(self) -> bool:
        return self._partial

    @partial_read.setter
    def partial_read(self, v: bool) -> None:
        if not self._wo:
            self._partial = bool(v)

    @property
    def write(self) -> bool:
        return self._write

    @write.setter
    def write(self, v: bool) -> None:
        if not self._ro:
            self._write = bool(v)

    @property
    def write_all(self) -> bool:
        return self._write_all

    @write_all.setter
    def write_all(self, v: bool) -> None:
        if not self._ro:
            self._write_all = bool(v)

    @property
    def read_only(self) -> bool:
        return self._ro

    @read_only.setter
    def read_only(self, v: bool) -> None:
        if v and not self._wo:
            self._write = False
            self._write_all = False
            self._wo = False
            self._ro = True
        elif not v:
            self._ro = False

    @property
    def write_only(self) -> bool:
        return self._wo

    @write_only.setter
    def write_only(self, v: bool) -> None:
        if v and not self._ro:
            self._read = False
            self._partial = False
            self._ro = False
            self._wo = True
        elif not v:
            self._wo = False

    # camelCase aliases for users of the reference API
    partialRead = partial_read
    writeAll = write_all
    readOnly = read_only
    writeOnly = write_only

    @property
    def zeroCopy(self) -> bool:  # noqa: N802
        return self.zero_copy

    @zeroCopy.setter
    def zeroCopy(self, v: bool) -> None:  # noqa: N802
        self.zero_copy = bool(v)

    @property
    def numberOfElementsPerWorkItem(self) -> int:  # noqa: N802
        return self.elements_per_work_item

    @numberOfElementsPerWorkItem.setter
    def numberOfElementsPerWorkItem(self, v: int) -> None:  # noqa: N802
        self.elements_per_work_item = int(v)

    @property
    def alignmentBytes(self) -> int:  # noqa: N802
        return self.alignment_bytes

    @property
    def gather(self) -> bool:
        """Alias of :attr:`gather_resident` (the ``gather`` readWrite token)."""
        return self.gather_resident

    @gather.setter
    def gather(self, v: bool) -> None:
        self.gather_resident = bool(v)

    gatherResident = gather

    # ------------------------------------------------------------ native spec
    def _spec(self, pin: bool = False):
        """``pin``: register wrapped host memory of any size (a compute
        captured into a graph replays its copies against the captured pages,
        which must be pinned)."""
        # The native spec is cached per (storage uid, flags): the uid changes
        # whenever the host storage does, so the pointer inside stays valid.
        key = (self._uid, self._read, self._partial, self._write, self._write_all, self._ro, self._wo,
               self.zero_copy, self.elements_per_work_item, self.elements_per_group, self.gather_resident, pin,
               None if self.blob_slices is None else tuple(self.blob_slices))
        cached = getattr(self, "_spec_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        arr = self.array
        moves = self._read or self._partial or self._write or self._write_all
        if self._fast is None and not self._registered and (
                self.zero_copy or (moves and (pin or arr.nbytes >= ClArray.auto_pin_min_bytes > 0))):
            # Page-lock wrapped host memory on first use (the reference pins
            # every array for each compute, Cores.cs:535-541): a copy from
            # pageable memory is staged by the runtime and a D2H blocks the
            # host until the stream drains, which defeats enqueue mode.
            # Refcounted per pointer in the native layer; released on
            # dispose / GC.  Device-only arrays (no transfer flag) stay as
            # they are (pinning would commit their untouched pages).
            self._registered = bool(cek.host_register(arr.ctypes.data, arr.nbytes))
        # zero-copy only when the GPU can map the memory (pinned FastArr or a
        # successful registration); otherwise the array is copied as usual
        zc = bool(self.zero_copy) and (self._fast is not None or self._registered)
        spec = cek.ArraySpec(self._uid, arr.ctypes.data, arr.nbytes, arr.itemsize,
                             self._read, self._partial, self._write, self._write_all,
                             self._ro, self._wo, zc, int(self.elements_per_work_item),
                             int(self.elements_per_group), bool(self.gather_resident))
        if self.blob_slices is not None:
            spec.blob_begin = [int(b) for b, _ in self.blob_slices]
            spec.blob_count = [int(n) for _, n in self.blob_slices]
        self._spec_cache = (key, spec)
        return spec

    @property
    def uid(self) -> int:
        return self._uid

    # ------------------------------------------------------------ chaining/API
    def next_param(self, *arrays) -> "ClParameterGroup":
        """Chain kernel parameters: ``a.next_param(b, c)`` → (a, b, c)."""
        g = ClParameterGroup([self])
        return g.next_param(*arrays)

    nextParam = next_param

    def compute(self, cruncher, compute_id: int, kernels: str, global_range: int, local_range: int = 256,
                global_offset: int = 0, pipeline: bool = False, pipeline_type: bool = True,
                pipeline_blobs: int = 4, granularity: int = 0) -> None:
        ClParameterGroup([self]).compute(cruncher, compute_id, kernels, global_range, local_range,
                                         global_offset, pipeline, pipeline_type, pipeline_blobs,
                                         granularity)

    def task(self, compute_id: int, kernels: str, global_range: int, local_range: int = 256,
             global_offset: int = 0, pipeline: bool = False, pipeline_type: bool = True,
             pipeline_blobs: int = 4):
        return ClParameterGroup([self]).task(compute_id, kernels, global_range, local_range,
                                             global_offset, pipeline, pipeline_type, pipeline_blobs)

    # ----------------------------------------------------------------- dispose
    def _release_device(self) -> None:
        _release_uid(self._uid)
        if self._registered:
            try:
                cek.host_unregister(self.array.ctypes.data)
            except Exception:
                pass
            self._registered = False

    @property
    def pinned(self) -> bool:
        """Host storage is page-locked (a FastArr, or registered wrapped memory)."""
        return (self._fast is not None and self._fast.pinned) or self._registered

    @property
    def is_deleted(self) -> bool:
        return self._disposed

    isDeleted = is_deleted

    def dispose(self) -> None:
        if self._disposed:
            return
        self._disposed = True
        try:
            self._release_device()
        finally:
            if self._fast is not None:
                self._fast.dispose()

    def __del__(self):
        try:
            if not self._disposed:
                _release_uid(self._uid)
                if self._registered and self._np is not None:
                    cek.host_unregister(self._np.ctypes.data)
        except Exception:
            pass

    def __repr__(self) -> str:
        flags = [n for n, v in (("partial", self._partial), ("read", self._read), ("write", self._write),
                                ("all", self._write_all), ("ro", self._ro), ("wo", self._wo),
                                ("zc", self.zero_copy)) if v]
        kind = "fast" if self._fast is not None else "host"
        return f"<ClArray n={self.N} dtype={self.dtype} {kind} [{' '.join(flags)}] epw={self.elements_per_work_item}>"


def as_clarray(x) -> ClArray:
    if isinstance(x, ClArray):
        return x
    return ClArray(x)


# --------------------------------------------------------------------------- groups


class ClParameterGroup:
    """Ordered kernel parameters (reference ``ClParameterGroup``)."""

    def __init__(self, arrays: Iterable = ()):
        self.arrays: list[ClArray] = [as_clarray(a) for a in arrays]

    @property
    def selected_arrays(self) -> list:
        return self.arrays

    selectedArrays = selected_arrays

    def next_param(self, *arrays) -> "ClParameterGroup":
        flat = []
        for a in arrays:
            if isinstance(a, ClParameterGroup):
                flat.extend(a.arrays)
            elif isinstance(a, (list, tuple)) and a and not np.isscalar(a[0]):
                flat.extend(as_clarray(x) for x in a)
            else:
                flat.append(as_clarray(a))
        return ClParameterGroup(self.arrays + flat)

    nextParam = next_param

    def __len__(self) -> int:
        return len(self.arrays)

    def __iter__(self):
        return iter(self.arrays)

    def compute(self, cruncher, compute_id: int, kernels: str, global_range: int, local_range: int = 256,
                global_offset: int = 0, pipeline: bool = False, pipeline_type: bool = True,
                pipeline_blobs: int = 4, granularity: int = 0) -> None:
        """Run ``kernels`` over ``global_range`` work items split across the
        cruncher's devices (ClArray.cs:543).  ``granularity`` (an extension)
        makes every device range a multiple of that many work items."""
        cruncher._compute_group(self, compute_id, kernels, global_range, local_range, global_offset,
                                pipeline, pipeline_type, pipeline_blobs, granularity=granularity)

    def task(self, compute_id: int, kernels: str, global_range: int, local_range: int = 256,
             global_offset: int = 0, pipeline: bool = False, pipeline_type: bool = True,
             pipeline_blobs: int = 4):
        """Freeze this compute (arrays + current flags) into a ClTask for task
        pools (reference ``task()``, ClArray.cs:515, :1552-1583)."""
        from .parallel.pool import ClTask

        return ClTask(self, compute_id, kernels, global_range, local_range, global_offset, pipeline,
                      pipeline_type, pipeline_blobs)

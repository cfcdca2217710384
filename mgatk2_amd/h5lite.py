"""Minimal h5py-style access to libhdf5 through ctypes.

h5py is not installed in this image, but the HDF5 C library is
(/opt/conda/lib/libhdf5.so, 1.10.x). This module covers the part of the h5py
API that the HDF5 writer (src/file_io/writers.py:60-406) and the QC report use:

* ``File(path, "w"|"r", libver=...)``, ``create_group``, ``create_dataset``
  (``data``, ``chunks``, ``compression="gzip"``, ``compression_opts``), ``attrs``;
* reading: ``f[name][...]`` / ``np.asarray(f[name])``, ``keys()``, ``attrs``.

Types are stored the way h5py stores them: numeric numpy dtypes as
little-endian standard types, ``S<n>`` as fixed-length NULLPAD ASCII strings,
Python ``str`` attributes as variable-length UTF-8 scalars, Python ints as
int64 and floats as float64 scalars.

Large 2-D gzip datasets are written chunk by chunk with ``H5Dwrite_chunk``
after a parallel deflate of all chunks (libmgphost.so ``mgp_deflate_tiles``),
which gives the same file content as libhdf5's single-threaded filter pipeline.
"""

from __future__ import annotations

import ctypes as C
import ctypes.util
import errno
import logging
import os
import time

import numpy as np

hid_t = C.c_int64
herr_t = C.c_int
hsize_t = C.c_uint64
H5P_DEFAULT = 0
H5S_ALL = 0
H5F_ACC_RDONLY, H5F_ACC_TRUNC = 0, 2
H5F_LIBVER_EARLIEST, H5F_LIBVER_LATEST = 0, 2
H5S_SCALAR = 0
H5T_INTEGER, H5T_FLOAT, H5T_STRING = 0, 1, 3
H5T_STR_NULLTERM, H5T_STR_NULLPAD = 0, 1
H5T_CSET_ASCII, H5T_CSET_UTF8 = 0, 1
H5I_GROUP, H5I_DATASET = 2, 5
H5_INDEX_NAME, H5_ITER_INC = 0, 0
H5T_VARIABLE = C.c_size_t(-1).value

_CANDIDATES = [os.environ.get("MGP_HDF5_LIB"), "/opt/conda/lib/libhdf5.so.103", "/opt/conda/lib/libhdf5.so",
               ctypes.util.find_library("hdf5")]
_lib = None
_T: dict[str, int] = {}


def available() -> bool:
    try:
        _h5()
        return True
    except OSError:
        return False


def _h5():
    global _lib
    if _lib is not None:
        return _lib
    err = None
    for cand in _CANDIDATES:
        if not cand:
            continue
        try:
            lib = C.CDLL(cand, use_errno=True)  # (errno of a failed write: _ck_retry)
            break
        except OSError as e:
            err = e
    else:
        raise OSError(f"libhdf5 not found (set MGP_HDF5_LIB): {err}")
    if lib.H5open() < 0:
        raise OSError("H5open failed")
    sig = {
        "H5Fcreate": (hid_t, [C.c_char_p, C.c_uint, hid_t, hid_t]),
        "H5Fopen": (hid_t, [C.c_char_p, C.c_uint, hid_t]),
        "H5Fclose": (herr_t, [hid_t]),
        "H5Fflush": (herr_t, [hid_t, C.c_int]),
        "H5Pcreate": (hid_t, [hid_t]),
        "H5Pclose": (herr_t, [hid_t]),
        "H5Pset_libver_bounds": (herr_t, [hid_t, C.c_int, C.c_int]),
        "H5Pset_chunk": (herr_t, [hid_t, C.c_int, C.POINTER(hsize_t)]),
        "H5Pset_deflate": (herr_t, [hid_t, C.c_uint]),
        "H5Screate": (hid_t, [C.c_int]),
        "H5Screate_simple": (hid_t, [C.c_int, C.POINTER(hsize_t), C.POINTER(hsize_t)]),
        "H5Sclose": (herr_t, [hid_t]),
        "H5Sget_simple_extent_ndims": (C.c_int, [hid_t]),
        "H5Sget_simple_extent_dims": (C.c_int, [hid_t, C.POINTER(hsize_t), C.POINTER(hsize_t)]),
        "H5Tcopy": (hid_t, [hid_t]),
        "H5Tclose": (herr_t, [hid_t]),
        "H5Tset_size": (herr_t, [hid_t, C.c_size_t]),
        "H5Tset_strpad": (herr_t, [hid_t, C.c_int]),
        "H5Tset_cset": (herr_t, [hid_t, C.c_int]),
        "H5Tget_class": (C.c_int, [hid_t]),
        "H5Tget_size": (C.c_size_t, [hid_t]),
        "H5Tget_sign": (C.c_int, [hid_t]),
        "H5Tis_variable_str": (C.c_int, [hid_t]),
        "H5Dcreate2": (hid_t, [hid_t, C.c_char_p, hid_t, hid_t, hid_t, hid_t, hid_t]),
        "H5Dopen2": (hid_t, [hid_t, C.c_char_p, hid_t]),
        "H5Dclose": (herr_t, [hid_t]),
        "H5Dwrite": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, C.c_void_p]),
        "H5Dread": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, C.c_void_p]),
        "H5Dwrite_chunk": (herr_t, [hid_t, hid_t, C.c_uint32, C.POINTER(hsize_t), C.c_size_t, C.c_void_p]),
        "H5Dget_space": (hid_t, [hid_t]),
        "H5Dget_type": (hid_t, [hid_t]),
        "H5Dget_create_plist": (hid_t, [hid_t]),
        "H5Pget_chunk": (C.c_int, [hid_t, C.c_int, C.POINTER(hsize_t)]),
        "H5Pget_nfilters": (C.c_int, [hid_t]),
        "H5Gcreate2": (hid_t, [hid_t, C.c_char_p, hid_t, hid_t, hid_t]),
        "H5Gopen2": (hid_t, [hid_t, C.c_char_p, hid_t]),
        "H5Gclose": (herr_t, [hid_t]),
        "H5Oopen": (hid_t, [hid_t, C.c_char_p, hid_t]),
        "H5Oclose": (herr_t, [hid_t]),
        "H5Iget_type": (C.c_int, [hid_t]),
        "H5Lexists": (C.c_int, [hid_t, C.c_char_p, hid_t]),
        "H5Lget_name_by_idx": (C.c_ssize_t, [hid_t, C.c_char_p, C.c_int, C.c_int, hsize_t, C.c_char_p, C.c_size_t,
                                             hid_t]),
        "H5Acreate2": (hid_t, [hid_t, C.c_char_p, hid_t, hid_t, hid_t, hid_t]),
        "H5Aopen": (hid_t, [hid_t, C.c_char_p, hid_t]),
        "H5Aclose": (herr_t, [hid_t]),
        "H5Awrite": (herr_t, [hid_t, hid_t, C.c_void_p]),
        "H5Aread": (herr_t, [hid_t, hid_t, C.c_void_p]),
        "H5Aget_type": (hid_t, [hid_t]),
        "H5Aget_space": (hid_t, [hid_t]),
        "H5Aexists": (C.c_int, [hid_t, C.c_char_p]),
        "H5Adelete": (herr_t, [hid_t, C.c_char_p]),
        "H5Aget_num_attrs": (C.c_int, [hid_t]),
        "H5Aget_name_by_idx": (C.c_ssize_t, [hid_t, C.c_char_p, C.c_int, C.c_int, hsize_t, C.c_char_p, C.c_size_t,
                                             hid_t]),
        "H5free_memory": (herr_t, [C.c_void_p]),
        "H5Gget_info": (herr_t, [hid_t, C.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    for n in ["H5P_CLS_FILE_ACCESS_ID_g", "H5P_CLS_DATASET_CREATE_ID_g", "H5T_C_S1_g",
              "H5T_STD_I8LE_g", "H5T_STD_U8LE_g", "H5T_STD_I16LE_g", "H5T_STD_U16LE_g", "H5T_STD_I32LE_g",
              "H5T_STD_U32LE_g", "H5T_STD_I64LE_g", "H5T_STD_U64LE_g", "H5T_IEEE_F32LE_g", "H5T_IEEE_F64LE_g"]:
        _T[n] = hid_t.in_dll(lib, n).value
    _lib = lib
    return lib


def _ck(v, what):
    if v < 0:
        raise OSError(f"HDF5 call failed: {what}")
    return v


# The reference's retry policy for writes and flushes on network filesystems
# (writers.py:23-26, _write_batch_with_retry / _flush_with_retry :266-323): a call that
# fails with EAGAIN is retried up to MAX_RETRIES times in all, sleeping 0.1 s, doubled
# per attempt up to 5 s; any other failure (or the last EAGAIN) raises at once.
MAX_RETRIES = 5
INITIAL_RETRY_DELAY = 0.1
MAX_RETRY_DELAY = 5.0
logger = logging.getLogger(__name__)
write_error_count = 0  # EAGAIN failures seen (the reference's write_error_count)


def _ck_retry(call, what, sleep=time.sleep):
    """Run ``call()`` (a libhdf5 call returning herr_t / hid_t) with the reference's
    EAGAIN retry and exponential backoff."""
    global write_error_count
    delay = INITIAL_RETRY_DELAY
    for attempt in range(MAX_RETRIES):
        C.set_errno(0)
        v = call()
        if v >= 0:
            if attempt > 0:
                logger.info("%s succeeded on attempt %d", what, attempt + 1)
            return v
        e = C.get_errno()
        if e != errno.EAGAIN:
            raise OSError(e or errno.EIO, f"HDF5 call failed: {what}")
        write_error_count += 1
        if attempt == MAX_RETRIES - 1:
            logger.error("%s failed after %d attempts", what, MAX_RETRIES)
            raise OSError(errno.EAGAIN, f"HDF5 call failed after {MAX_RETRIES} attempts: {what}")
        logger.warning("Temporary write error (attempt %d/%d), retrying in %.2fs: %s", attempt + 1, MAX_RETRIES,
                       delay, what)
        sleep(delay)
        delay = min(delay * 2, MAX_RETRY_DELAY)
    raise AssertionError("unreachable")


_NUM = {
    np.dtype("int8"): "H5T_STD_I8LE_g", np.dtype("uint8"): "H5T_STD_U8LE_g",
    np.dtype("int16"): "H5T_STD_I16LE_g", np.dtype("uint16"): "H5T_STD_U16LE_g",
    np.dtype("int32"): "H5T_STD_I32LE_g", np.dtype("uint32"): "H5T_STD_U32LE_g",
    np.dtype("int64"): "H5T_STD_I64LE_g", np.dtype("uint64"): "H5T_STD_U64LE_g",
    np.dtype("float32"): "H5T_IEEE_F32LE_g", np.dtype("float64"): "H5T_IEEE_F64LE_g",
}


def _type_for(dt: np.dtype) -> tuple[int, bool]:
    """(HDF5 type id, owned) for a numpy dtype."""
    lib = _h5()
    dt = np.dtype(dt)
    if dt.kind == "S":
        t = _ck(lib.H5Tcopy(_T["H5T_C_S1_g"]), "H5Tcopy")
        lib.H5Tset_size(t, max(1, dt.itemsize))
        lib.H5Tset_strpad(t, H5T_STR_NULLPAD)
        lib.H5Tset_cset(t, H5T_CSET_ASCII)
        return t, True
    if dt.newbyteorder("<") in _NUM and dt.byteorder in ("=", "<", "|"):
        return _T[_NUM[dt.newbyteorder("<")]], False
    raise TypeError(f"unsupported dtype {dt}")


def _vlen_str_type() -> int:
    lib = _h5()
    t = _ck(lib.H5Tcopy(_T["H5T_C_S1_g"]), "H5Tcopy")
    lib.H5Tset_size(t, H5T_VARIABLE)
    lib.H5Tset_cset(t, H5T_CSET_UTF8)
    return t


def _dims(shape) -> C.Array:
    return (hsize_t * max(1, len(shape)))(*shape)


def _space(shape) -> int:
    lib = _h5()
    if len(shape) == 0:
        return _ck(lib.H5Screate(H5S_SCALAR), "H5Screate")
    return _ck(lib.H5Screate_simple(len(shape), _dims(shape), None), "H5Screate_simple")


def _shape_of(space: int) -> tuple[int, ...]:
    lib = _h5()
    nd = lib.H5Sget_simple_extent_ndims(space)
    if nd <= 0:
        return ()
    d = (hsize_t * nd)()
    lib.H5Sget_simple_extent_dims(space, d, None)
    return tuple(int(x) for x in d)


def _dtype_of(t: int) -> np.dtype | str:
    lib = _h5()
    cls = lib.H5Tget_class(t)
    size = lib.H5Tget_size(t)
    if cls == H5T_INTEGER:
        return np.dtype(("i" if lib.H5Tget_sign(t) == 1 else "u") + str(size)).newbyteorder("<")
    if cls == H5T_FLOAT:
        return np.dtype("f" + str(size)).newbyteorder("<")
    if cls == H5T_STRING:
        return "vlen" if lib.H5Tis_variable_str(t) > 0 else np.dtype(f"S{size}")
    raise TypeError(f"unsupported HDF5 type class {cls}")


def _read_vlen_strings(reader, obj: int, count: int) -> list[str]:
    lib = _h5()
    t = _vlen_str_type()
    ptrs = (C.c_char_p * max(1, count))()
    try:
        _ck(reader(obj, t, ptrs), "read vlen string")
        return [(p or b"").decode("utf-8") for p in ptrs[:count]]
    finally:
        lib.H5Tclose(t)


class _GInfo(C.Structure):  # H5G_info_t
    _fields_ = [("storage_type", C.c_int), ("nlinks", hsize_t), ("max_corder", C.c_int64), ("mounted", C.c_bool)]


class Attrs:
    def __init__(self, oid: int):
        self._id = oid

    def __setitem__(self, name: str, value):
        lib = _h5()
        if lib.H5Aexists(self._id, name.encode()) > 0:
            lib.H5Adelete(self._id, name.encode())
        if isinstance(value, str):
            t, own = _vlen_str_type(), True
            sp = _space(())
            buf = (C.c_char_p * 1)(value.encode("utf-8"))
            a = _ck(lib.H5Acreate2(self._id, name.encode(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "H5Acreate2")
            try:
                _ck(lib.H5Awrite(a, t, buf), "H5Awrite")
            finally:
                lib.H5Aclose(a)
                lib.H5Sclose(sp)
                lib.H5Tclose(t)
            return
        arr = np.asarray(value)
        if arr.dtype == np.bool_:
            arr = arr.astype(np.uint8)
        if arr.dtype.kind == "U":
            arr = arr.astype("S")
        arr = np.require(arr, requirements='C')
        t, own = _type_for(arr.dtype)
        sp = _space(arr.shape)
        a = _ck(lib.H5Acreate2(self._id, name.encode(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "H5Acreate2")
        try:
            _ck(lib.H5Awrite(a, t, arr.ctypes.data), "H5Awrite")
        finally:
            lib.H5Aclose(a)
            lib.H5Sclose(sp)
            if own:
                lib.H5Tclose(t)

    def __getitem__(self, name: str):
        lib = _h5()
        if lib.H5Aexists(self._id, name.encode()) <= 0:
            raise KeyError(name)
        a = _ck(lib.H5Aopen(self._id, name.encode(), H5P_DEFAULT), "H5Aopen")
        t = lib.H5Aget_type(a)
        sp = lib.H5Aget_space(a)
        try:
            shape = _shape_of(sp)
            dt = _dtype_of(t)
            n = int(np.prod(shape)) if shape else 1
            if dt == "vlen":
                vals = _read_vlen_strings(lib.H5Aread, a, n)
                return vals[0] if not shape else np.array(vals, dtype=object).reshape(shape)
            out = np.empty(shape, dt)
            mt, own = _type_for(dt)
            _ck(lib.H5Aread(a, mt, out.ctypes.data), "H5Aread")
            if own:
                lib.H5Tclose(mt)
            return out[()] if not shape else out
        finally:
            lib.H5Sclose(sp)
            lib.H5Tclose(t)
            lib.H5Aclose(a)

    def keys(self):
        lib = _h5()
        out = []
        for i in range(lib.H5Aget_num_attrs(self._id)):
            buf = C.create_string_buffer(1024)
            lib.H5Aget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, 1024, H5P_DEFAULT)
            out.append(buf.value.decode())
        return out

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def __contains__(self, name):
        return _h5().H5Aexists(self._id, name.encode()) > 0


class Dataset:
    def __init__(self, did: int, name: str):
        self._id = did
        self.name = name
        lib = _h5()
        sp = lib.H5Dget_space(did)
        t = lib.H5Dget_type(did)
        self.shape = _shape_of(sp)
        self._dt = _dtype_of(t)
        self.dtype = np.dtype(object) if self._dt == "vlen" else self._dt
        lib.H5Sclose(sp)
        lib.H5Tclose(t)
        self.attrs = Attrs(did)

    @property
    def chunks(self):
        lib = _h5()
        p = lib.H5Dget_create_plist(self._id)
        try:
            d = (hsize_t * 8)()
            nd = lib.H5Pget_chunk(p, 8, d)
            return tuple(int(x) for x in d[:nd]) if nd > 0 else None
        finally:
            lib.H5Pclose(p)

    @property
    def compression(self):
        lib = _h5()
        p = lib.H5Dget_create_plist(self._id)
        try:
            return "gzip" if lib.H5Pget_nfilters(p) > 0 else None
        finally:
            lib.H5Pclose(p)

    def read(self) -> np.ndarray:
        lib = _h5()
        n = int(np.prod(self.shape)) if self.shape else 1
        if self._dt == "vlen":
            return np.array(_read_vlen_strings(lambda o, t, b: lib.H5Dread(o, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, b),
                                               self._id, n), dtype=object).reshape(self.shape)
        out = np.empty(self.shape, self._dt)
        mt, own = _type_for(self._dt)
        try:
            if n:
                _ck(lib.H5Dread(self._id, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.ctypes.data), "H5Dread")
        finally:
            if own:
                lib.H5Tclose(mt)
        return out

    def __getitem__(self, key):
        return self.read()[key]

    def __array__(self, dtype=None, copy=None):
        a = self.read()
        return a if dtype is None else a.astype(dtype)

    def __len__(self):
        return self.shape[0]

    def close(self):
        if self._id is not None:
            _h5().H5Dclose(self._id)
            self._id = None


class Group:
    def __init__(self, gid: int, name: str = "/"):
        self._id = gid
        self.name = name
        self.attrs = Attrs(gid)
        self._children: list = []

    def create_group(self, name: str) -> Group:
        lib = _h5()
        g = Group(_ck(lib.H5Gcreate2(self._id, name.encode(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), "H5Gcreate2"),
                  name)
        self._children.append(g)
        return g

    def create_dataset(self, name: str, data=None, chunks=None, compression=None, compression_opts=None,
                       shape=None, dtype=None, n_threads: int = 0):
        lib = _h5()
        arr = np.asarray(data) if data is not None else np.zeros(shape, dtype)
        if arr.dtype.kind == "U":
            arr = arr.astype("S")
        if arr.dtype == np.bool_:
            arr = arr.astype(np.uint8)
        arr = np.require(arr, requirements='C')
        level = None
        if compression == "gzip" or isinstance(compression, int):
            level = compression_opts if compression_opts is not None else (compression if isinstance(compression, int)
                                                                           else 4)
        if level is not None and chunks is None:
            chunks = tuple(max(1, min(s, 1 << 14)) for s in arr.shape) if arr.shape else None
        t, own = _type_for(arr.dtype)
        sp = _space(arr.shape)
        dcpl = H5P_DEFAULT
        try:
            if chunks and arr.shape and all(s > 0 for s in arr.shape):
                dcpl = _ck(lib.H5Pcreate(_T["H5P_CLS_DATASET_CREATE_ID_g"]), "H5Pcreate")
                _ck(lib.H5Pset_chunk(dcpl, len(chunks), _dims(chunks)), "H5Pset_chunk")
                if level is not None:
                    _ck(lib.H5Pset_deflate(dcpl, int(level)), "H5Pset_deflate")
            did = _ck(lib.H5Dcreate2(self._id, name.encode(), t, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT), "H5Dcreate2")
            try:
                if arr.size:
                    if dcpl != H5P_DEFAULT and level is not None and arr.ndim == 2:
                        self._write_chunks(did, arr, chunks, int(level), n_threads)
                    else:
                        _ck_retry(lambda: lib.H5Dwrite(did, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.ctypes.data),
                                  "H5Dwrite")
            except Exception:
                lib.H5Dclose(did)
                raise
        finally:
            if dcpl != H5P_DEFAULT:
                lib.H5Pclose(dcpl)
            lib.H5Sclose(sp)
            if own:
                lib.H5Tclose(t)
        ds = Dataset(did, name)
        self._children.append(ds)
        return ds

    def create_dataset_from_chunks(self, name: str, shape, dtype, chunks, level: int, tiles: list[bytes]):
        """A chunked gzip dataset written from already deflated chunks (the
        H5Z_DEFLATE form, row-major over the chunk grid: mgp_h5_plane_tiles, or
        mgp_h5_tiles on the device as u8 arrays)."""
        lib = _h5()
        t, own = _type_for(np.dtype(dtype))
        sp = _space(shape)
        dcpl = _ck(lib.H5Pcreate(_T["H5P_CLS_DATASET_CREATE_ID_g"]), "H5Pcreate")
        try:
            _ck(lib.H5Pset_chunk(dcpl, len(chunks), _dims(chunks)), "H5Pset_chunk")
            _ck(lib.H5Pset_deflate(dcpl, int(level)), "H5Pset_deflate")
            did = _ck(lib.H5Dcreate2(self._id, name.encode(), t, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT), "H5Dcreate2")
            try:
                nc = -(-shape[1] // chunks[1])
                off = (hsize_t * 2)()
                for i, blob in enumerate(tiles):
                    off[0] = (i // nc) * chunks[0]
                    off[1] = (i % nc) * chunks[1]
                    # (bytes, or a u8 array view: Engine.h5_tiles)
                    ptr = blob.ctypes.data if isinstance(blob, np.ndarray) else blob
                    _ck_retry(lambda: lib.H5Dwrite_chunk(did, H5P_DEFAULT, 0, off, len(blob), ptr),
                              "H5Dwrite_chunk")
            except Exception:
                lib.H5Dclose(did)
                raise
        finally:
            lib.H5Pclose(dcpl)
            lib.H5Sclose(sp)
            if own:
                lib.H5Tclose(t)
        ds = Dataset(did, name)
        self._children.append(ds)
        return ds

    @staticmethod
    def _write_chunks(did: int, arr: np.ndarray, chunks, level: int, n_threads: int):
        from .bam import deflate_tiles

        lib = _h5()
        tiles = deflate_tiles(arr, (int(chunks[0]), int(chunks[1])), level=level, n_threads=n_threads)
        nc = -(-arr.shape[1] // chunks[1])
        off = (hsize_t * 2)()
        for i, blob in enumerate(tiles):
            off[0] = (i // nc) * chunks[0]
            off[1] = (i % nc) * chunks[1]
            _ck_retry(lambda: lib.H5Dwrite_chunk(did, H5P_DEFAULT, 0, off, len(blob), blob), "H5Dwrite_chunk")

    def __contains__(self, name: str) -> bool:
        return _h5().H5Lexists(self._id, name.encode(), H5P_DEFAULT) > 0

    def keys(self) -> list[str]:
        lib = _h5()
        info = _GInfo()
        _ck(lib.H5Gget_info(self._id, C.byref(info)), "H5Gget_info")
        out = []
        for i in range(int(info.nlinks)):
            buf = C.create_string_buffer(1024)
            _ck(lib.H5Lget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, 1024, H5P_DEFAULT),
                "H5Lget_name_by_idx")
            out.append(buf.value.decode())
        return out

    def __iter__(self):
        return iter(self.keys())

    def __getitem__(self, name: str):
        lib = _h5()
        if not name in self:  # noqa: E713
            raise KeyError(name)
        o = _ck(lib.H5Oopen(self._id, name.encode(), H5P_DEFAULT), "H5Oopen")
        kind = lib.H5Iget_type(o)
        lib.H5Oclose(o)
        if kind == H5I_DATASET:
            ds = Dataset(_ck(lib.H5Dopen2(self._id, name.encode(), H5P_DEFAULT), "H5Dopen2"), name)
            self._children.append(ds)
            return ds
        if kind == H5I_GROUP:
            g = Group(_ck(lib.H5Gopen2(self._id, name.encode(), H5P_DEFAULT), "H5Gopen2"), name)
            self._children.append(g)
            return g
        raise KeyError(name)

    def _close_children(self):
        lib = _h5()
        for ch in self._children:
            if isinstance(ch, Dataset):
                ch.close()
            elif ch._id is not None:
                ch._close_children()
                lib.H5Gclose(ch._id)
                ch._id = None
        self._children = []


class File(Group):
    def __init__(self, path, mode: str = "r", libver=None):
        lib = _h5()
        self.filename = str(path)
        self._writable = mode in ("w", "w-", "x")
        if mode in ("w", "w-", "x"):
            fapl = _ck(lib.H5Pcreate(_T["H5P_CLS_FILE_ACCESS_ID_g"]), "H5Pcreate")
            if libver == "latest":
                lib.H5Pset_libver_bounds(fapl, H5F_LIBVER_LATEST, H5F_LIBVER_LATEST)
            fid = lib.H5Fcreate(str(path).encode(), H5F_ACC_TRUNC, H5P_DEFAULT, fapl)
            lib.H5Pclose(fapl)
        elif mode == "r":
            fid = lib.H5Fopen(str(path).encode(), H5F_ACC_RDONLY, H5P_DEFAULT)
        else:
            raise ValueError(f"unsupported mode {mode}")
        if fid < 0:
            raise OSError(f"cannot open HDF5 file {path}")
        self._fid = fid
        root = _ck(lib.H5Gopen2(fid, b"/", H5P_DEFAULT), "H5Gopen2")
        super().__init__(root, "/")

    def close(self):
        if getattr(self, "_fid", None) is None:
            return
        lib = _h5()
        self._close_children()
        lib.H5Gclose(self._id)
        fid = self._fid
        try:
            if self._writable:
                _ck_retry(lambda: lib.H5Fflush(fid, 0), "H5Fflush")  # (H5F_SCOPE_LOCAL)
        finally:  # the file id is released (and its lock dropped) even when the flush fails
            self._fid = None
            self._id = None
            lib.H5Fclose(fid)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def module():
    """An h5py-like namespace (``.File``) for the writers."""

    class _M:
        pass

    m = _M()
    m.File = File
    return m


__all__ = ["File", "Group", "Dataset", "available", "module"]

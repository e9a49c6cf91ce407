"""ctypes wrapper over oracle/_build/liboracle_cms.so (the C restatement).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by mahout_amd/ (the product).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle_cms.so")

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    if not os.path.exists(_SO):
        build()
    lib = ctypes.CDLL(_SO)
    c = ctypes
    sig = {
        "orc_hash_params": (None, [c.c_int64, c.c_int32, _i64p, _i64p]),
        "orc_hash": (c.c_int32, [c.c_int64, c.c_int64, c.c_int32, c.c_int64]),
        "orc_hash_many": (None, [_i64p, _i64p, c.c_int32, c.c_int32, _i64p, c.c_int64, _i32p]),
        "orc_shape_from_delta_epsilon": (c.c_int, [c.c_double, c.c_double, c.POINTER(c.c_int32), c.POINTER(c.c_int32)]),
        "orc_sketch_build": (None, [_f64p, c.c_int64, c.c_int32, c.c_int32, _i64p, _i64p, _i64p, _i64p, c.c_void_p, c.c_int64]),
        "orc_sketch_get": (c.c_double, [c.c_void_p, c.c_int32, c.c_int32, _i64p, _i64p, c.c_int64]),
        "orc_sketch_cosine": (c.c_double, [c.c_void_p, c.c_void_p, c.c_int32, c.c_int32]),
        "orc_normalize_weight_result": (c.c_double, [c.c_double, c.c_int, c.c_int, c.c_int]),
        "orc_cosine_cm": (c.c_double, [c.c_void_p, c.c_void_p, c.c_int32, c.c_int32, c.c_int]),
        "orc_similarities_row": (None, [_f64p, c.c_int64, c.c_int32, c.c_int32, c.c_int64, c.c_int, _f64p]),
        "orc_top_users": (c.c_int32, [_i64p, _f64p, c.c_int64, c.c_int32, _i64p, _f64p]),
        "orc_estimate_preference": (c.c_float, [_f64p, c.c_int32, c.c_int32, _i64p, _i64p, c.c_int64, _i64p, c.c_int64,
                                                c.c_int64, c.c_int, c.c_int, c.c_float, c.c_float]),
        "orc_fmeasure": (c.c_double, [c.c_int32, c.c_int32, c.c_int32, c.c_int32, c.c_double]),
        "orc_compute_config": (c.c_int, [c.c_int32, c.c_int32, c.c_double, c.POINTER(c.c_int32), c.POINTER(c.c_int32),
                                         c.POINTER(c.c_double), c.POINTER(c.c_double)]),
        "orc_faithful_pairs": (c.c_int64, [_i64p, _i64p, c.c_void_p, c.c_int64, c.c_int32, c.c_int32, _i64p, _i64p,
                                           _i64p, _i64p, c.c_int64, _f64p]),
        "orc_build_rows_reuse": (c.c_int64, [_i64p, _i64p, c.c_void_p, c.c_int64, c.c_int64, c.c_int32, c.c_int32,
                                             _i64p, _i64p, c.POINTER(c.c_double)]),
        "orc_ingest_faithful_par": (c.c_int64, [_i64p, _i64p, c.c_void_p, c.c_int64, c.c_int64, c.c_int32, c.c_int32,
                                                _i64p, _i64p, c.c_int32, c.POINTER(c.c_double)]),
        "orc_ingest_efficient_par": (c.c_int64, [_i64p, _i64p, c.c_void_p, c.c_int64, c.c_int64, c.c_int32,
                                                 c.c_int32, _i64p, _i64p, c.c_int32, c.c_void_p,
                                                 c.POINTER(c.c_double)]),
        "orc_faithful_pairs_par": (c.c_int64, [_i64p, _i64p, c.c_void_p, c.c_int64, c.c_int32, c.c_int32, _i64p,
                                               _i64p, _i64p, _i64p, c.c_int64, c.c_int32, c.POINTER(c.c_double)]),
        "orc_allpairs_efficient_par": (c.c_int64, [_f64p, c.c_int64, c.c_int32, c.c_int32, c.c_int64, c.c_int64,
                                                   c.c_int32, c.POINTER(c.c_double)]),
        "orc_max_threads": (c.c_int32, []),
        "orc_recommend_par": (c.c_int64, [_f64p, c.c_int64, c.c_int32, c.c_int32, _i64p, _i64p, _i64p, _i32p, _i64p,
                                          c.c_int64, c.c_int32, c.c_int32, c.c_int32, c.c_float, c.c_float, c.c_int64,
                                          c.c_int64, c.c_int32, c.POINTER(c.c_double)]),
        "orc_per_owner_rows_csr": (None, [_i64p, _i64p, c.c_int64, _i32p, _i32p, _i64p, _i64p, _i64p, c.c_int64,
                                          c.c_int32, _f64p]),
        "orc_cosine_queries_csr": (None, [_f64p, c.c_int64, _i64p, _i64p, c.c_void_p, c.c_int64, c.c_int32, c.c_int32,
                                          _i64p, _i64p, c.c_int, c.c_int32, _f64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _vp(arr):
    return None if arr is None else arr.ctypes.data_as(ctypes.c_void_p)


def hash_params(seed, depth):
    a = np.zeros(depth, np.int64)
    b = np.zeros(depth, np.int64)
    lib().orc_hash_params(seed, depth, a, b)
    return a, b


def hash_keys(a, b, width, keys):
    keys = np.ascontiguousarray(keys, np.int64)
    out = np.zeros((keys.size, len(a)), np.int32)
    lib().orc_hash_many(np.ascontiguousarray(a, np.int64), np.ascontiguousarray(b, np.int64), len(a), width,
                        keys, keys.size, out)
    return out


def shape_from_delta_epsilon(delta, epsilon):
    w = ctypes.c_int32()
    d = ctypes.c_int32()
    rc = lib().orc_shape_from_delta_epsilon(delta, epsilon, ctypes.byref(w), ctypes.byref(d))
    if rc != 0:
        raise ValueError("CMException: delta/epsilon out of range")
    return w.value, d.value


def build_table(rows, depth, width, a, b, owner_row, key, val=None):
    """fp64 [rows][depth][width] table, updates applied in stream order."""
    table = np.zeros((rows, depth, width), np.float64)
    owner_row = np.ascontiguousarray(owner_row, np.int64)
    key = np.ascontiguousarray(key, np.int64)
    v = None if val is None else np.ascontiguousarray(val, np.float32)
    lib().orc_sketch_build(table, rows, depth, width, a, b, owner_row, key, _vp(v), owner_row.size)
    return table


def sketch_get(sketch, a, b, key):
    sk = np.ascontiguousarray(sketch, np.float64)
    d, w = sk.shape
    return lib().orc_sketch_get(_vp(sk), d, w, a, b, int(key))


def cosine(sa, sb):
    sa = np.ascontiguousarray(sa, np.float64)
    sb = np.ascontiguousarray(sb, np.float64)
    d, w = sa.shape
    return lib().orc_sketch_cosine(_vp(sa), _vp(sb), d, w)


def cosine_cm(sa, sb, weighted=False):
    sa = np.ascontiguousarray(sa, np.float64)
    sb = np.ascontiguousarray(sb, np.float64)
    d, w = sa.shape
    return lib().orc_cosine_cm(_vp(sa), _vp(sb), d, w, int(weighted))


def normalize_weight_result(r, count=1, num=0, weighted=False):
    return lib().orc_normalize_weight_result(r, count, num, int(weighted))


def similarities_row(table, q, weighted=False):
    rows, d, w = table.shape
    out = np.zeros(rows, np.float64)
    lib().orc_similarities_row(np.ascontiguousarray(table), rows, d, w, q, int(weighted), out)
    return out


def estimate_preference(table, a, b, user_row, nb_rows, item_key, weighted=False, capper=None):
    """GenericUserBasedRecommender.doEstimatePreference with the CosineCM point
    query; capper = (min, max) or None."""
    rows, d, w = table.shape
    nb = np.ascontiguousarray(nb_rows, np.int64)
    lo, hi = capper if capper is not None else (0.0, 0.0)
    return lib().orc_estimate_preference(np.ascontiguousarray(table), d, w, np.ascontiguousarray(a, np.int64),
                                         np.ascontiguousarray(b, np.int64), int(user_row), nb, nb.size,
                                         int(item_key), int(weighted), int(capper is not None), float(lo), float(hi))


def cosine_queries_csr(qsk, off, keys, vals, depth, width, a, b, weighted=False, threads=16):
    """userSimilarity of each query sketch (qsk [Q][d][w] fp64) with EVERY
    owner of the CSR (off [n+1], keys, vals or None), the owners' sketch rows
    taken from their keys (orc_cosine_queries_csr): [Q][n] fp64."""
    qsk = np.ascontiguousarray(qsk, dtype=np.float64).reshape(-1, depth * width)
    off = np.ascontiguousarray(off, dtype=np.int64)
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    n = off.size - 1
    vals = None if vals is None else np.ascontiguousarray(vals, dtype=np.float32)
    out = np.empty((qsk.shape[0], n), np.float64)
    lib().orc_cosine_queries_csr(qsk, qsk.shape[0], off, keys, _vp(vals), n, depth, width, a, b, int(weighted),
                                 int(threads), out)
    return out


def top_users(ids, scores, k):
    ids = np.ascontiguousarray(ids, np.int64)
    scores = np.ascontiguousarray(scores, np.float64)
    oi = np.zeros(k, np.int64)
    os_ = np.zeros(k, np.float64)
    n = lib().orc_top_users(ids, scores, ids.size, k, oi, os_)
    return oi[:n], os_[:n]


def fmeasure(w, d, n, u, q):
    return lib().orc_fmeasure(w, d, n, u, q)


def compute_config(n_prefs, u_items, q):
    w = ctypes.c_int32()
    d = ctypes.c_int32()
    de = ctypes.c_double()
    ep = ctypes.c_double()
    rc = lib().orc_compute_config(n_prefs, u_items, q, ctypes.byref(w), ctypes.byref(d), ctypes.byref(de),
                                  ctypes.byref(ep))
    if rc != 0:
        raise RuntimeError("No solution found")
    return w.value, d.value, de.value, ep.value


def faithful_pairs(offsets, keys, vals, rows, depth, width, a, b, pi, pj):
    out = np.zeros(len(pi), np.float64)
    v = None if vals is None else np.ascontiguousarray(vals, np.float32)
    lib().orc_faithful_pairs(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(keys, np.int64), _vp(v),
                             rows, depth, width, a, b, np.ascontiguousarray(pi, np.int64),
                             np.ascontiguousarray(pj, np.int64), len(pi), out)
    return out


def build_rows_reuse(offsets, keys, vals, lo, hi, depth, width, a, b):
    cs = ctypes.c_double()
    v = None if vals is None else np.ascontiguousarray(vals, np.float32)
    n = lib().orc_build_rows_reuse(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(keys, np.int64),
                                   _vp(v), lo, hi, depth, width, a, b, ctypes.byref(cs))
    return n, cs.value


# ---- per-owner shapes (CountMinSketchConfig + CosineCM), composed from the
# restated primitives above.  Test infrastructure only.

def owner_config(offsets, u_items, q):
    """CountMinSketchConfig.computeConfig (T/impl/common/CountMinSketchConfig.java:120-158)
    for every owner: (delta, epsilon) arrays; n = the owner's preference count."""
    offsets = np.asarray(offsets, np.int64)
    n = offsets.size - 1
    de = np.zeros(n, np.float64)
    ep = np.zeros(n, np.float64)
    for r in range(n):
        _, _, de[r], ep[r] = compute_config(int(offsets[r + 1] - offsets[r]), int(u_items), float(q))
    return de, ep


def owner_shapes(delta, epsilon):
    """AbstractCountMinSketch(delta, epsilon) shape per owner; (0, 0) for CMException."""
    w = np.zeros(len(delta), np.int32)
    d = np.zeros(len(delta), np.int32)
    for r, (de, ep) in enumerate(zip(delta, epsilon)):
        try:
            w[r], d[r] = shape_from_delta_epsilon(float(de), float(ep))
        except ValueError:
            pass
    return w, d


def export_profile(offsets, keys, vals, row, width, depth, a, b):
    """CosineCM.exportProfile(row, delta, epsilon) (T/impl/similarity/CosineCM.java:41-58):
    a fresh [depth][width] sketch of the owner's preferences, in their order."""
    lo, hi = int(offsets[row]), int(offsets[row + 1])
    v = None if vals is None else np.asarray(vals, np.float32)[lo:hi]
    k = np.asarray(keys, np.int64)[lo:hi]
    return build_table(1, depth, width, a, b, np.zeros(hi - lo, np.int64), k, v)[0]


def per_owner_similarity(offsets, keys, vals, shapes, a, b, u1, u2, weighted=False):
    """CosineCM.userSimilarity(u1, u2) (CosineCM.java:83-96): u1's sketch built
    with u2's (delta, epsilon), against u2's own sketch."""
    w, d = int(shapes[0][u2]), int(shapes[1][u2])
    if w == 0:
        raise ValueError("CMException")
    s1 = export_profile(offsets, keys, vals, u1, w, d, a, b)
    s2 = export_profile(offsets, keys, vals, u2, w, d, a, b)
    return cosine_cm(s1, s2, weighted)


def per_owner_rows_csr(offsets, keys, shapes, a, b, queries, threads=16):
    """per_owner_similarity(offsets, keys, None, shapes, a, b, u1, u2) for
    every u1 in queries (<= 64) and EVERY owner u2 (sparse rows, grouped by
    shape; orc_per_owner_rows_csr): [len(queries)][n] float64."""
    off = np.ascontiguousarray(offsets, np.int64)
    n = off.size - 1
    q = np.ascontiguousarray(queries, np.int64)
    if q.size > 64:
        raise ValueError("at most 64 queries per call")
    out = np.zeros((q.size, n), np.float64)
    lib().orc_per_owner_rows_csr(off, np.ascontiguousarray(keys, np.int64), n,
                                 np.ascontiguousarray(shapes[0], np.int32), np.ascontiguousarray(shapes[1], np.int32),
                                 np.ascontiguousarray(a, np.int64), np.ascontiguousarray(b, np.int64), q, q.size,
                                 int(threads), out)
    return out


# ---- CPU baselines (oracle/cms_baseline.c; bench.py's cpu_baseline legs) ----

def max_threads():
    return lib().orc_max_threads()


def ingest_faithful(offsets, keys, vals, lo, hi, depth, width, a, b, threads):
    v = None if vals is None else np.ascontiguousarray(vals, np.float32)
    cs = ctypes.c_double()
    n = lib().orc_ingest_faithful_par(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(keys, np.int64),
                                      _vp(v), lo, hi, depth, width, np.ascontiguousarray(a, np.int64),
                                      np.ascontiguousarray(b, np.int64), threads, ctypes.byref(cs))
    return n, cs.value


def ingest_efficient(offsets, keys, vals, lo, hi, depth, width, a, b, threads, table=None):
    v = None if vals is None else np.ascontiguousarray(vals, np.float32)
    if table is None:
        table = np.empty((hi - lo) * depth * width, np.uint32)
    cs = ctypes.c_double()
    n = lib().orc_ingest_efficient_par(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(keys, np.int64),
                                       _vp(v), lo, hi, depth, width, np.ascontiguousarray(a, np.int64),
                                       np.ascontiguousarray(b, np.int64), threads, _vp(table), ctypes.byref(cs))
    return n, cs.value, table


def faithful_pairs_par(offsets, keys, vals, rows, depth, width, a, b, pi, pj, threads):
    v = None if vals is None else np.ascontiguousarray(vals, np.float32)
    cs = ctypes.c_double()
    n = lib().orc_faithful_pairs_par(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(keys, np.int64),
                                     _vp(v), rows, depth, width, np.ascontiguousarray(a, np.int64),
                                     np.ascontiguousarray(b, np.int64), np.ascontiguousarray(pi, np.int64),
                                     np.ascontiguousarray(pj, np.int64), len(pi), threads, ctypes.byref(cs))
    return n, cs.value


def allpairs_efficient(table, i_lo, i_hi, threads):
    t = np.ascontiguousarray(table, np.float64)
    rows, d, w = t.shape
    cs = ctypes.c_double()
    n = lib().orc_allpairs_efficient_par(t.reshape(-1), rows, d, w, i_lo, i_hi, threads, ctypes.byref(cs))
    return n, cs.value


def recommend_par(table, a, b, off, items, item_keys, nn, how_many, u_lo, u_hi, threads, capper=None):
    """orc_recommend_par: GenericUserBasedRecommender.recommend for users
    [u_lo, u_hi) over prebuilt sketches (efficient CPU mode); returns
    (estimates computed, checksum of the recommended values)."""
    t = np.ascontiguousarray(table, np.float64)
    rows, d, w = t.shape
    lo, hi = capper if capper is not None else (0.0, 0.0)
    cs = ctypes.c_double()
    n = lib().orc_recommend_par(t.reshape(-1), rows, d, w, np.ascontiguousarray(a, np.int64),
                                np.ascontiguousarray(b, np.int64), np.ascontiguousarray(off, np.int64),
                                np.ascontiguousarray(items, np.int32), np.ascontiguousarray(item_keys, np.int64),
                                len(item_keys), nn, how_many, int(capper is not None), float(lo), float(hi), u_lo, u_hi,
                                threads, ctypes.byref(cs))
    return n, cs.value

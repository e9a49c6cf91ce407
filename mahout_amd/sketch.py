"""SketchTable: a handle to the device-resident count-min-sketch table.

Thin, typed wrapper over the C ABI (include/mahout_cms.h).  One table holds
the [num_owners][depth][width] u32 sketches of every owner; the reference
builds the same sketches one DoubleCountMinSketch at a time
(T/impl/common/DoubleCountMinSketch.java, T/impl/similarity/CosineCM.java:41-67).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _dev_ptr(x):
    """Device pointer from an int or a torch tensor (None passes through)."""
    if x is None:
        return None
    if isinstance(x, int):
        return ctypes.c_void_p(x)
    return ctypes.c_void_p(x.data_ptr())


def _torch_stream(*xs):
    """Current torch stream (hipStream_t) of the first device tensor (0: the
    legacy default stream), or None when no input is a device tensor."""
    import torch

    for x in xs:
        if isinstance(x, torch.Tensor) and x.is_cuda:
            return torch.cuda.current_stream(x.device).cuda_stream
    return None


def shape_from_delta_epsilon(delta, epsilon):
    """AbstractCountMinSketch(delta, epsilon) shape rule -> (width, depth)."""
    lib = _lib.load()
    w = ctypes.c_int32()
    d = ctypes.c_int32()
    check(lib.cms_shape_from_delta_epsilon(delta, epsilon, ctypes.byref(w), ctypes.byref(d)))
    return w.value, d.value


def frac_bits_for(values, max_bits=31):
    """Smallest frac_bits with every value * 2^frac_bits an integer (the
    preference granularity a u32 handle needs); ValueError when none <= max_bits."""
    v = np.asarray(values, np.float32).astype(np.float64)
    if v.size == 0:
        return 0
    for fb in range(max_bits + 1):
        x = np.ldexp(v, fb)
        if np.all(x == np.floor(x)):
            return fb
    raise ValueError("preference values need more than %d fractional bits" % max_bits)


def shard_of_key(key, world):
    return _lib.load().cms_shard_of_key(int(key), int(world))


def comm_unique_id():
    buf = (ctypes.c_uint8 * 128)()
    check(_lib.load().cms_comm_unique_id(buf))
    return bytes(buf)


class SketchTable:
    def __init__(self, num_owners, depth=5, width=4096, seed=42, weighted=False, device=-1, owner_ids=None,
                 per_owner=False, frac_bits=0, counters="u32", collective_single_rank=False):
        """counters: "u32" (exact integer counters in units of 2^-frac_bits) or
        "f64" (DoubleCountMinSketch's fp64 counters for any float preference).
        collective_single_rank: CMS_FLAG_COLLECTIVE_SINGLE_RANK (a one-rank
        comm_init still takes the multi-rank data path)."""
        lib = _lib.load()
        p = _lib.CmsParams()
        check(lib.cms_params_init(ctypes.byref(p)))
        p.counter_type = {"u32": _lib.CMS_COUNTER_U32, "f64": _lib.CMS_COUNTER_F64}[counters]
        p.depth = depth
        p.width = width
        p.seed = seed
        p.num_owners = num_owners
        p.weighting = _lib.CMS_WEIGHTED if weighted else _lib.CMS_UNWEIGHTED
        p.device = device
        p.frac_bits = frac_bits
        p.flags = _lib.CMS_FLAG_COLLECTIVE_SINGLE_RANK if collective_single_rank else 0
        h = ctypes.c_void_p()
        create = lib.cms_create_per_owner if per_owner else lib.cms_create
        check(create(ctypes.byref(p), ctypes.byref(h)))
        self.per_owner = per_owner
        self.counters = counters
        self._lib = lib
        self._h = h
        if device < 0:  # the device the library chose (hipGetDevice at creation), not torch's guess
            device = self.stats()["device"]
        self.device = int(device)
        self.num_owners = num_owners
        self.depth = depth
        self.width = width
        self.seed = seed
        self.hash_rows = 32 if per_owner else depth  # CMS_MAX_DEPTH rows for per-owner handles
        if owner_ids is not None:
            self.set_owner_ids(owner_ids)

    # -- lifecycle --
    def close(self):
        if self._h:
            self._lib.cms_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- setup --
    def set_owner_ids(self, ids):
        ids = np.ascontiguousarray(ids, np.int64)
        check(self._lib.cms_set_owner_ids(self._h, _ptr(ids), ids.size))

    def hash_params(self):
        """(a_i, b_i) of every hash row: depth rows, or all CMS_MAX_DEPTH (32)
        rows of a per-owner handle (any owner's shape may use them)."""
        a = np.zeros(self.hash_rows, np.int64)
        b = np.zeros(self.hash_rows, np.int64)
        check(self._lib.cms_hash_params(self._h, _ptr(a), _ptr(b)))
        return a, b

    def set_hash_params(self, a, b):
        """Install a HashFunctionBuilder's drawn (a_i, b_i) (cms_set_hash_params);
        one pair per sketch row of the handle (32 for per-owner handles)."""
        a = np.ascontiguousarray(a, np.int64)
        b = np.ascontiguousarray(b, np.int64)
        if a.shape != b.shape:
            raise ValueError("a and b differ in length")
        check(self._lib.cms_set_hash_params(self._h, _ptr(a), _ptr(b), int(a.size)))

    def hash_keys(self, keys):
        keys = np.ascontiguousarray(keys, np.int64)
        out = np.zeros((keys.size, self.depth), np.int32)
        check(self._lib.cms_hash_keys(self._h, _ptr(keys), keys.size, _ptr(out)))
        return out

    # -- ingest --
    def ingest(self, owner, key, val=None):
        owner = np.ascontiguousarray(owner, np.int64)
        key = np.ascontiguousarray(key, np.int64)
        v = None if val is None else np.ascontiguousarray(val, np.float32)
        if owner.size != key.size or (v is not None and v.size != key.size):
            raise ValueError("owner/key/val length mismatch")
        check(self._lib.cms_ingest(self._h, _ptr(owner), _ptr(key), _ptr(v), owner.size))

    def ingest_device_rows(self, d_row, d_key, d_val, n):
        # stream-ordered both ways (no host wait): the library's stream waits
        # for the producers on torch's current stream, and torch's stream waits
        # for the ingest, so the inputs may be freed once this returns.  The
        # library stream is a blocking stream, so against torch's legacy
        # default stream (s == 0) that ordering is implicit.
        s = _torch_stream(d_row, d_key, d_val)
        if s:
            check(self._lib.cms_wait_stream(self._h, ctypes.c_void_p(s)))
        check(self._lib.cms_ingest_device_rows(self._h, _dev_ptr(d_row), _dev_ptr(d_key), _dev_ptr(d_val), int(n)))
        if s:
            check(self._lib.cms_release_to_stream(self._h, ctypes.c_void_p(s)))
        elif s is None:
            self.synchronize()

    def ingest_csr(self, offsets, keys, vals=None):
        offsets = np.ascontiguousarray(offsets, np.int64)
        keys = np.ascontiguousarray(keys, np.int64)
        v = None if vals is None else np.ascontiguousarray(vals, np.float32)
        if offsets.size != self.num_owners + 1:
            raise ValueError("offsets must have num_owners + 1 entries")
        check(self._lib.cms_ingest_csr(self._h, _ptr(offsets), _ptr(keys), _ptr(v)))

    def ingest_csr_device(self, d_offsets, d_keys, d_vals=None):
        s = _torch_stream(d_offsets, d_keys, d_vals)
        if s:
            check(self._lib.cms_wait_stream(self._h, ctypes.c_void_p(s)))
        check(self._lib.cms_ingest_csr_device(self._h, _dev_ptr(d_offsets), _dev_ptr(d_keys), _dev_ptr(d_vals)))
        if s:
            check(self._lib.cms_release_to_stream(self._h, ctypes.c_void_p(s)))
        elif s is None:
            self.synchronize()

    def reset(self):
        check(self._lib.cms_reset(self._h))

    def comm_init(self, unique_id, rank, world):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        check(self._lib.cms_comm_init(self._h, buf, rank, world))

    def comm_init_transport(self, rank, world, allreduce, allgather):
        """cms_comm_init_transport: a caller-supplied communicator in place of
        RCCL.  allreduce(d_ptr, count) sums `count` u64 words at device address
        d_ptr over all ranks in place; allgather(d_send, d_recv, nbytes) writes
        every rank's `nbytes` bytes at d_send, in rank order, to d_recv.  See
        mahout_amd.transport for a torch.distributed implementation."""
        def ar(ptr, count, _user):
            try:
                allreduce(int(ptr), int(count))
                return 0
            except Exception:  # noqa: BLE001 -- reported as a status code
                import traceback
                traceback.print_exc()
                return 1

        def ag(send, recv, nbytes, _user):
            try:
                allgather(int(send), int(recv), int(nbytes))
                return 0
            except Exception:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1
        # the C side keeps the function pointers: hold the thunks for the handle's life
        self._transport = (_lib.ALLREDUCE_FN(ar), _lib.ALLGATHER_FN(ag))
        check(self._lib.cms_comm_init_transport(self._h, int(rank), int(world), self._transport[0],
                                                self._transport[1], None))

    def finalize(self):
        check(self._lib.cms_finalize(self._h))

    def finalize_with(self, allreduce):
        """cms_finalize_with: merge through a caller collective.
        allreduce(d_ptr, count) must sum `count` u64 words at device address
        d_ptr over all ranks, in place."""
        def thunk(ptr, count, _user):
            try:
                allreduce(int(ptr), int(count))
                return 0
            except Exception:  # noqa: BLE001 -- reported as a status code
                import traceback
                traceback.print_exc()
                return 1
        cb = _lib.ALLREDUCE_FN(thunk)
        check(self._lib.cms_finalize_with(self._h, cb, None))

    def synchronize(self):
        check(self._lib.cms_synchronize(self._h))

    # -- queries --
    def similarity(self, id1, id2):
        out = ctypes.c_double()
        check(self._lib.cms_similarity(self._h, int(id1), int(id2), ctypes.byref(out)))
        return out.value

    def similarities(self, id1, ids2):
        ids2 = np.ascontiguousarray(ids2, np.int64)
        out = np.zeros(ids2.size, np.float64)
        check(self._lib.cms_similarities(self._h, int(id1), _ptr(ids2), ids2.size, _ptr(out)))
        return out

    def point_query(self, owner_id, key):
        out = ctypes.c_double()
        check(self._lib.cms_point_query(self._h, int(owner_id), int(key), ctypes.byref(out)))
        return out.value

    def most_similar(self, owner_id, k):
        ids = np.zeros(k, np.int64)
        sc = np.zeros(k, np.float64)
        cnt = ctypes.c_int32()
        check(self._lib.cms_most_similar(self._h, int(owner_id), int(k), _ptr(ids), _ptr(sc), ctypes.byref(cnt)))
        return ids[:cnt.value], sc[:cnt.value]

    def top_k_rows(self, row_begin, row_count, k):
        ids = np.zeros((row_count, k), np.int64)
        sc = np.zeros((row_count, k), np.float64)
        cnt = np.zeros(row_count, np.int32)
        check(self._lib.cms_top_k_rows(self._h, int(row_begin), int(row_count), int(k), _ptr(ids), _ptr(sc),
                                       _ptr(cnt)))
        return ids, sc, cnt

    def estimate_preferences(self, user_id, neighbor_ids, item_keys, capper=None):
        """doEstimatePreference(user, neighbourhood, item) for every item key
        (CosineCM point-query path); capper = (min, max) or None."""
        nb = np.ascontiguousarray(neighbor_ids, np.int64)
        it = np.ascontiguousarray(item_keys, np.int64)
        out = np.zeros(it.size, np.float32)
        lo, hi = capper if capper is not None else (0.0, 0.0)
        check(self._lib.cms_estimate_preferences(self._h, int(user_id), _ptr(nb), nb.size, _ptr(it), it.size,
                                                 int(capper is not None), float(lo), float(hi), _ptr(out)))
        return out

    def estimate_preferences_batch(self, user_ids, nb_offsets, neighbor_ids, item_offsets, item_keys, capper=None):
        """estimate_preferences for many users in one call
        (cms_estimate_preferences_batch): user u's neighbourhood is
        neighbor_ids[nb_offsets[u]:nb_offsets[u+1]], its candidates
        item_keys[item_offsets[u]:item_offsets[u+1]]; returns one float32
        estimate per candidate."""
        us = np.ascontiguousarray(user_ids, np.int64)
        nbo = np.ascontiguousarray(nb_offsets, np.int64)
        nb = np.ascontiguousarray(neighbor_ids, np.int64)
        ito = np.ascontiguousarray(item_offsets, np.int64)
        it = np.ascontiguousarray(item_keys, np.int64)
        if nbo.size != us.size + 1 or ito.size != us.size + 1:
            raise ValueError("offset arrays need len(user_ids) + 1 entries")
        # the library reads neighbor_ids / item_keys up to the last offsets and
        # writes item_offsets[-1] estimates: the offsets must describe exactly
        # these arrays, or the call would run past the host buffers
        for name, o, arr in (("nb_offsets", nbo, nb), ("item_offsets", ito, it)):
            if o[0] != 0 or o[-1] != arr.size or (o.size > 1 and bool(np.any(np.diff(o) < 0))):
                raise ValueError(f"{name} must start at 0, never decrease and end at the length of its array")
        out = np.zeros(it.size, np.float32)
        lo, hi = capper if capper is not None else (0.0, 0.0)
        check(self._lib.cms_estimate_preferences_batch(self._h, us.size, _ptr(us), _ptr(nbo), _ptr(nb), _ptr(ito),
                                                       _ptr(it), int(capper is not None), float(lo), float(hi),
                                                       _ptr(out)))
        return out

    def recommend_batch(self, user_ids, nb_offsets, neighbor_ids, model_user_ids, pref_offsets, pref_items,
                        how_many, include_known=False, capper=None):
        """cms_recommend_batch: GenericUserBasedRecommender.recommend for every
        user of user_ids at once. User u's neighbourhood is
        neighbor_ids[nb_offsets[u]:nb_offsets[u+1]] (IDs); the DataModel is
        model_user_ids (ascending) with row r's item IDs
        pref_items[pref_offsets[r]:pref_offsets[r+1]]. Returns (counts [n],
        items [n][how_many], values [n][how_many] float32)."""
        us = np.ascontiguousarray(user_ids, np.int64)
        nbo = np.ascontiguousarray(nb_offsets, np.int64)
        nb = np.ascontiguousarray(neighbor_ids, np.int64)
        mu = np.ascontiguousarray(model_user_ids, np.int64)
        po = np.ascontiguousarray(pref_offsets, np.int64)
        pi = np.ascontiguousarray(pref_items, np.int64)
        # the library reads every array up to its last offset: they must match
        if nbo.size != us.size + 1 or nbo[0] != 0 or nbo[-1] != nb.size or bool(np.any(np.diff(nbo) < 0)):
            raise ValueError("nb_offsets must hold len(user_ids) + 1 non-decreasing entries from 0 to len(neighbor_ids)")
        if po.size != mu.size + 1 or po[0] != 0 or po[-1] != pi.size or bool(np.any(np.diff(po) < 0)):
            raise ValueError("pref_offsets must hold len(model_user_ids) + 1 non-decreasing entries from 0 to "
                             "len(pref_items)")
        if how_many < 1:
            raise ValueError("howMany must be at least 1")
        counts = np.zeros(us.size, np.int32)
        items = np.full((us.size, how_many), -1, np.int64)
        vals = np.full((us.size, how_many), np.nan, np.float32)
        lo, hi = capper if capper is not None else (0.0, 0.0)
        check(self._lib.cms_recommend_batch(self._h, us.size, _ptr(us), _ptr(nbo), _ptr(nb), mu.size, _ptr(mu),
                                            _ptr(po), _ptr(pi), int(how_many), int(bool(include_known)),
                                            int(capper is not None), float(lo), float(hi), _ptr(counts),
                                            _ptr(items), _ptr(vals)))
        return counts, items, vals

    def write_similar_items(self, path, k, as_float=True):
        """cms_top_k_all in FileSimilarItemsWriter's CSV format."""
        check(self._lib.cms_write_similar_items(self._h, os.fsencode(path), int(k), int(as_float)))

    def write_similarities(self, path, k, fmt, threshold=None):
        """cms_write_similarities: fmt 'item_similarity_job' (MR ItemSimilarityJob
        text result) or 'spark_itemsimilarity' (TextDelimitedIndexedDatasetWriter);
        threshold: RowSimilarityJob's --threshold (cms_write_similarities_threshold)."""
        code = {"item_similarity_job": _lib.CMS_FORMAT_ITEM_SIMILARITY_JOB,
                "spark_itemsimilarity": _lib.CMS_FORMAT_SPARK_ITEMSIMILARITY}[fmt]
        if threshold is None:
            check(self._lib.cms_write_similarities(self._h, os.fsencode(path), int(k), code))
        else:
            check(self._lib.cms_write_similarities_threshold(self._h, os.fsencode(path), int(k), code,
                                                             float(threshold)))

    def top_k_all_partial(self, k, shard, nshards):
        n = self.num_owners
        ids = np.zeros((n, k), np.int64)
        sc = np.zeros((n, k), np.float64)
        cnt = np.zeros(n, np.int32)
        check(self._lib.cms_top_k_all_partial(self._h, int(k), int(shard), int(nshards), _ptr(ids), _ptr(sc),
                                              _ptr(cnt)))
        return ids, sc, cnt

    def top_k_merge(self, k, parts):
        """parts: list of (ids, scores, counts) partial lists."""
        n = self.num_owners
        ids = np.ascontiguousarray(np.stack([p[0] for p in parts]), np.int64)
        sc = np.ascontiguousarray(np.stack([p[1] for p in parts]), np.float64)
        cnt = np.ascontiguousarray(np.stack([p[2] for p in parts]), np.int32)
        oi = np.zeros((n, k), np.int64)
        os_ = np.zeros((n, k), np.float64)
        oc = np.zeros(n, np.int32)
        check(self._lib.cms_top_k_merge(self._h, int(k), len(parts), _ptr(ids), _ptr(sc), _ptr(cnt), _ptr(oi),
                                        _ptr(os_), _ptr(oc)))
        return oi, os_, oc

    def top_k_all(self, k):
        """mostSimilar lists of every owner, [num_owners][k] by owner row
        (symmetric streaming all-pairs pass)."""
        n = self.num_owners
        # uninitialised on purpose: the library defines every cell (ID -1 and a
        # NaN score past a row's count)
        ids = np.empty((n, k), np.int64)
        sc = np.empty((n, k), np.float64)
        cnt = np.empty(n, np.int32)
        check(self._lib.cms_top_k_all(self._h, int(k), _ptr(ids), _ptr(sc), _ptr(cnt)))
        return ids, sc, cnt

    def _device_lists(self, k):
        import torch
        dev = torch.device("cuda", self.device)
        n = self.num_owners
        return (torch.empty((n, k), dtype=torch.int64, device=dev), torch.empty((n, k), dtype=torch.float64, device=dev),
                torch.empty(n, dtype=torch.int32, device=dev))

    def top_k_all_device(self, k):
        """top_k_all(k) with the lists left on the handle's GPU as torch
        tensors (cms_top_k_all_device): (ids [n][k], scores [n][k], counts [n])."""
        out = self._device_lists(k)
        check(self._lib.cms_top_k_all_device(self._h, int(k), *[ctypes.c_void_p(x.data_ptr()) for x in out]))
        return out

    def top_k_refresh_device(self, k):
        """top_k_refresh(k) into device tensors (cms_top_k_refresh_device)."""
        out = self._device_lists(k)
        check(self._lib.cms_top_k_refresh_device(self._h, int(k), *[ctypes.c_void_p(x.data_ptr()) for x in out]))
        return out

    def top_k_refresh(self, k):
        """The same lists as top_k_all(k), recomputing only the pairs with an
        owner touched by COO ingests since the previous refresh (the first
        call runs the whole job and keeps 2k-deep lists on the device)."""
        n = self.num_owners
        ids = np.empty((n, k), np.int64)
        sc = np.empty((n, k), np.float64)
        cnt = np.empty(n, np.int32)
        check(self._lib.cms_top_k_refresh(self._h, int(k), _ptr(ids), _ptr(sc), _ptr(cnt)))
        return ids, sc, cnt

    def refresh_stats(self):
        """(owners touched, lists recomputed whole, whole jobs) of the last refresh."""
        v = [ctypes.c_int64(0) for _ in range(3)]
        check(self._lib.cms_refresh_stats(self._h, *[ctypes.byref(x) for x in v]))
        return tuple(int(x.value) for x in v)

    def refresh_classes(self):
        """{class: (owners, touched)} of the last refresh's job, classes
        "multi" (multi-limb), "int8" and "fp4" (cms_refresh_classes)."""
        v = (ctypes.c_int64 * 6)()
        check(self._lib.cms_refresh_classes(self._h, v))
        return {c: (int(v[i]), int(v[3 + i])) for i, c in enumerate(("multi", "int8", "fp4"))}

    # -- per-owner shapes (CountMinSketchConfig) --
    @classmethod
    def per_owner_shapes(cls, num_owners, seed=42, weighted=False, device=-1, owner_ids=None, frac_bits=0):
        """A handle whose owners each carry their own (d, w): CosineCM with
        its CountMinSketchConfig (cms_create_per_owner)."""
        return cls(num_owners, seed=seed, weighted=weighted, device=device, owner_ids=owner_ids, per_owner=True,
                   frac_bits=frac_bits)

    def configure_owner_shapes(self, q, num_keys):
        """CountMinSketchConfig(q).configure(dataModel) on the GPU."""
        check(self._lib.cms_configure_owner_shapes(self._h, float(q), int(num_keys)))

    def set_owner_delta_epsilon(self, delta, epsilon):
        de = np.ascontiguousarray(delta, np.float64)
        ep = np.ascontiguousarray(epsilon, np.float64)
        if de.size != self.num_owners or ep.size != self.num_owners:
            raise ValueError("one (delta, epsilon) per owner")
        check(self._lib.cms_set_owner_delta_epsilon(self._h, _ptr(de), _ptr(ep)))

    def owner_shapes(self):
        """(delta, epsilon, width, depth) per owner row."""
        n = self.num_owners
        de, ep = np.zeros(n, np.float64), np.zeros(n, np.float64)
        w, d = np.zeros(n, np.int32), np.zeros(n, np.int32)
        check(self._lib.cms_get_owner_shapes(self._h, _ptr(de), _ptr(ep), _ptr(w), _ptr(d)))
        return de, ep, w, d

    def read_owner_sketch(self, owner_id):
        """getExportedCMProfile(owner_id): [depth][width] fp64."""
        w = ctypes.c_int32()
        d = ctypes.c_int32()
        check(self._lib.cms_read_owner_sketch(self._h, int(owner_id), None, 0, ctypes.byref(w), ctypes.byref(d)))
        out = np.zeros((d.value, w.value), np.float64)
        check(self._lib.cms_read_owner_sketch(self._h, int(owner_id), _ptr(out), out.size, ctypes.byref(w),
                                              ctypes.byref(d)))
        return out

    def read_counters(self, row_begin=0, row_count=None):
        if row_count is None:
            row_count = self.num_owners - row_begin
        out = np.zeros((row_count, self.depth, self.width), np.float64)
        check(self._lib.cms_read_counters(self._h, int(row_begin), int(row_count), _ptr(out)))
        return out

    FORMS = ("u32", "u16", "u8", "u4", "u2", "u1", "list")

    def owner_forms(self, row_begin=0, row_count=None):
        """(form code per owner -- an index into FORMS --, the counter bound
        each narrow form was chosen for) of owners [row_begin, +row_count)
        (cms_owner_forms)."""
        if row_count is None:
            row_count = self.num_owners - row_begin
        form = np.zeros(row_count, np.int32)
        bound = np.zeros(row_count, np.uint32)
        check(self._lib.cms_owner_forms(self._h, int(row_begin), int(row_count), _ptr(form), _ptr(bound)))
        return form, bound

    def read_counters_device(self, row_begin=0, row_count=None, out=None):
        """Counters [row_count][d][w] on the handle's device, in counter units
        (cms_read_counters_device).  The tensor is torch.int32 holding the u32
        bits (torch's integer reductions work on it); a counter at or above
        2^31 reads negative -- use .view(torch.uint32) or mask with 0xFFFFFFFF
        in int64 where such counters can occur."""
        import torch
        if row_count is None:
            row_count = self.num_owners - row_begin
        if out is None:
            out = torch.empty((row_count, self.depth, self.width), dtype=torch.int32,
                              device=torch.device("cuda", self.device))
        if out.device != torch.device("cuda", self.device) or out.element_size() != 4 or not out.is_contiguous():
            raise ValueError("out must be a contiguous 4-byte tensor on cuda:%d" % self.device)
        if out.numel() < row_count * self.depth * self.width:
            raise ValueError("out holds fewer than row_count * depth * width counters")
        check(self._lib.cms_read_counters_device(self._h, int(row_begin), int(row_count), ctypes.c_void_p(out.data_ptr())))
        s = torch.cuda.current_stream(out.device).cuda_stream
        if s:  # later torch work on this stream waits for the copy
            check(self._lib.cms_release_to_stream(self._h, ctypes.c_void_p(s)))
        return out

    def release_scratch(self):
        """cms_release_scratch: ingest/query scratch and the kept refresh lists
        go back to the allocator (the next refresh is a whole job)."""
        check(self._lib.cms_release_scratch(self._h))

    # -- instrumentation --
    def stats(self):
        s = _lib.CmsStats()
        s.struct_size = ctypes.sizeof(s)
        check(self._lib.cms_get_stats(self._h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in s._fields_}

    def set_timing(self, enabled=True, level=2):
        """HIP-event timing of the library's kernel scopes.  level 1 brackets
        only the roofline kernels (cheap enough for timed steps), level 2 every
        phase scope as well (each event costs the stream a few us)."""
        check(self._lib.cms_set_timing(self._h, int(level) if enabled else 0))

    def timing(self, name):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._lib.cms_get_timing(self._h, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def reset_timing(self):
        check(self._lib.cms_reset_timing(self._h))


def shard_of_keys(keys, world):
    """Vectorised cms_shard_of_key (splitmix64 finalizer mod world) for host
    arrays -- used to route a stream's pairs to their rank before ingest."""
    z = np.asarray(keys, np.int64).astype(np.uint64)
    if world <= 1:
        return np.zeros(z.shape, np.int32)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world)).astype(np.int32)


def java_double_to_string(v):
    """Java Double.toString(v) as the library writes it (cms_format_java_double)."""
    buf = ctypes.create_string_buffer(64)
    n = _lib.load().cms_format_java_double(float(v), buf, 64)
    if n < 0:
        raise ValueError(v)
    return buf.value.decode()

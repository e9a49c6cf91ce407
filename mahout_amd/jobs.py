"""Driver replacements for the distributed similarity surfaces the north star
names: the MapReduce ItemSimilarityJob and
spark-itemsimilarity, run with the sketch cosine (CosineCM's measure) on the
GPU instead of their own co-occurrence pipelines.

Neither reference driver can host this measure as a plugin:
- ItemSimilarityJob's pluggable VectorSimilarityMeasure
  (mr/.../math/hadoop/similarity/cooccurrence/measures/VectorSimilarityMeasure.java:22-33)
  scores a pair from the dot product of two item vectors and their norms;
  CosineCM's min over d sketch rows of per-row cosines
  (DoubleCountMinSketch.java:114-149) is not such a function.
- spark-itemsimilarity computes LLR over A'A only
  (math-scala/.../cf/SimilarityAnalysis.scala:61-134) and has no measure
  plug point.
So these are drop-in *drivers*: the same command-line options, input
parsing and output files as the reference jobs
(T/hadoop/similarity/item/ItemSimilarityJob.java:97-183,
T/hadoop/ToEntityPrefsMapper.java:58-80, T/hadoop/item/ToUserVectorsReducer.java:66-80;
spark/.../drivers/ItemSimilarityDriver.scala, TextDelimitedReaderWriter.scala:244-303),
with the similarity computed by libmahout_cms.so.

What they deliberately do not reproduce:
- ItemSimilarityJob's --maxPrefs sampling (RowSimilarityJob samples rows and
  columns with more observations down at random, --randomSeed): a cost
  control of the co-occurrence pipeline.  The sketch path uses every
  preference, i.e. the reference's result with maxPrefs >= the largest row.
- Order among exactly equal similarities in a top list: the reference's
  Lucene PriorityQueue keeps whichever came first in hash-index order
  (unspecified); here ties keep the lower item ID (TopItems order).
- A repeated (user, item) line: the reference keeps the value its reducer
  saw last (arbitrary order); here the last line of the input wins.
"""
import os
import re

import numpy as np

from . import _lib
from .datamodel import java_parse_float, java_parse_long
from .sketch import SketchTable
from .taste import counter_units

SKETCH_COSINE = "SIMILARITY_COSINE_CM"  # --similarityClassname of the sketch measure
_DELIM = re.compile(r"[\t,]")  # ToEntityPrefsMapper.DELIMITER


def _input_files(path):
    """A file, or every visible file of a directory (Hadoop skips names
    starting with '_' or '.')."""
    if os.path.isdir(path):
        return [os.path.join(path, f) for f in sorted(os.listdir(path))
                if not f.startswith(("_", ".")) and os.path.isfile(os.path.join(path, f))]
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return [path]


def _java_split(pattern, line):
    """String.split(regex) / Pattern.split: trailing empty strings dropped."""
    tok = pattern.split(line)
    while tok and tok[-1] == "":
        tok.pop()
    return tok if tok else [""]


def read_item_prefs(path, boolean_data=False, min_prefs_per_user=1):
    """The item-user preference matrix of PreparePreferenceMatrixJob: lines
    `userID,itemID[,pref]` split on tab or comma, IDs Long.parseLong, the
    preference Float.parseFloat (1.0 when absent or with booleanData), users
    with fewer than min_prefs_per_user distinct items left out
    (ToUserVectorsReducer.java:76).  Returns (item_ids, offsets, user_keys,
    values) with items as owners, each owner's users ascending."""
    prefs = {}  # user -> {item: value}
    for fn in _input_files(path):
        with open(fn) as f:
            for line in f:
                tok = _java_split(_DELIM, line.rstrip("\n").rstrip("\r"))
                if len(tok) < 2:
                    raise ValueError(f"ArrayIndexOutOfBoundsException: line {line!r}")
                u, it = java_parse_long(tok[0]), java_parse_long(tok[1])
                v = 1.0 if boolean_data or len(tok) < 3 else float(java_parse_float(tok[2]))
                prefs.setdefault(u, {})[it] = v
    by_item = {}
    for u, row in prefs.items():
        if len(row) < min_prefs_per_user:
            continue
        for it, v in row.items():
            by_item.setdefault(it, {})[u] = v
    item_ids = np.array(sorted(by_item), np.int64)
    off = np.zeros(item_ids.size + 1, np.int64)
    keys, vals = [], []
    for r, it in enumerate(item_ids):
        row = by_item[int(it)]
        for u in sorted(row):
            keys.append(u)
            vals.append(row[u])
        off[r + 1] = len(keys)
    return item_ids, off, np.array(keys, np.int64), np.array(vals, np.float32)


def _sketch_table(item_ids, off, keys, vals, depth, width, seed, device):
    fb, counters = counter_units(off, vals)
    t = SketchTable(item_ids.size, depth=depth, width=width, seed=seed, device=device, owner_ids=item_ids,
                    frac_bits=fb, counters=counters)
    t.ingest_csr(off, keys, vals)
    t.finalize()
    return t


def _parse(args, spec):
    """AbstractJob-style `--name value` / `-short value` options."""
    out = {name: default for name, (_, default) in spec.items()}
    short = {s: name for name, (s, _) in spec.items() if s}
    i = 0
    while i < len(args):
        a = args[i]
        name = a[2:] if a.startswith("--") else short.get(a[1:]) if a.startswith("-") else None
        if name is None or name not in spec:
            raise ValueError(f"Unexpected argument {a!r}")
        if i + 1 >= len(args):
            raise ValueError(f"Missing value for {a}")
        out[name] = args[i + 1]
        i += 2
    return out


class ItemSimilarityJob:
    """org.apache.mahout.cf.taste.hadoop.similarity.item.ItemSimilarityJob with
    --similarityClassname SIMILARITY_COSINE_CM.  Output: <output>/part-r-00000
    with one `itemA<TAB>itemB<TAB>similarity` line per distinct pair of the
    per-item top lists, itemA < itemB, sorted (EntityEntityWritable order),
    similarity > Double.MIN_VALUE and >= --threshold, printed as
    Double.toString; plus an empty _SUCCESS marker."""

    DEFAULT_MAX_SIMILAR_ITEMS_PER_ITEM = 100
    DEFAULT_MAX_PREFS = 500
    DEFAULT_MIN_PREFS_PER_USER = 1
    SPEC = {
        "input": ("i", None), "output": ("o", None), "similarityClassname": ("s", None),
        "maxSimilaritiesPerItem": ("m", str(DEFAULT_MAX_SIMILAR_ITEMS_PER_ITEM)),
        "maxPrefs": ("mppu", str(DEFAULT_MAX_PREFS)),
        "minPrefsPerUser": ("mp", str(DEFAULT_MIN_PREFS_PER_USER)),
        "booleanData": ("b", "false"), "threshold": ("tr", None), "randomSeed": (None, None),
        "tempDir": (None, None), "startPhase": (None, None), "endPhase": (None, None),
        # sketch shape and HashFunctionBuilder seed of the measure
        "sketchDepth": (None, "5"), "sketchWidth": (None, "4096"), "hashSeed": (None, "42"),
    }

    def run(self, args, device=-1):
        o = _parse(list(args), self.SPEC)
        if o["input"] is None or o["output"] is None:
            raise ValueError("--input and --output are required")
        if o["similarityClassname"] != SKETCH_COSINE:
            raise ValueError(f"this driver computes {SKETCH_COSINE} only; the co-occurrence measures "
                             f"({o['similarityClassname']}) belong to the reference's RowSimilarityJob")
        k = int(o["maxSimilaritiesPerItem"])
        if k <= 0:
            raise ValueError("maxSimilarItemsPerItem must be greater then 0!")  # ItemSimilarityJob.java:196
        min_prefs = int(o["minPrefsPerUser"])
        boolean = o["booleanData"].lower() == "true"  # Boolean.valueOf
        thr = None if o["threshold"] is None else float(o["threshold"])
        items, off, keys, vals = read_item_prefs(o["input"], boolean, min_prefs)
        os.makedirs(o["output"], exist_ok=True)
        out = os.path.join(o["output"], "part-r-00000")
        if items.size == 0:
            open(out, "w").close()
        else:
            with _sketch_table(items, off, keys, vals, int(o["sketchDepth"]), int(o["sketchWidth"]),
                               int(o["hashSeed"]), device) as t:
                t.write_similarities(out, min(k, items.size), "item_similarity_job", threshold=thr)
        open(os.path.join(o["output"], "_SUCCESS"), "w").close()
        return 0


class ItemSimilarityDriver:
    """spark-itemsimilarity (org.apache.mahout.drivers.ItemSimilarityDriver)
    with the sketch cosine in place of LLR, for long IDs: input lines split
    by --inDelim (default "[,\\t ]"), --rowIDColumn / --itemIDColumn; output
    <output>/similarity-matrix/part-00000 in TextDelimitedIndexedDatasetWriter's
    default schema ("itemID<TAB>ID1:s1 ID2:s2 ...", strength descending)."""

    SPEC = {
        "input": ("i", None), "output": ("o", None), "maxSimilaritiesPerItem": ("m", "100"),
        "inDelim": (None, "[,\t ]"), "rowIDColumn": ("rc", "0"), "itemIDColumn": ("ic", "1"),
        "sketchDepth": (None, "5"), "sketchWidth": (None, "4096"), "hashSeed": (None, "42"),
    }

    def run(self, args, device=-1):
        o = _parse(list(args), self.SPEC)
        if o["input"] is None or o["output"] is None:
            raise ValueError("--input and --output are required")
        delim = re.compile(o["inDelim"])
        rc, ic = int(o["rowIDColumn"]), int(o["itemIDColumn"])
        by_item = {}
        for fn in _input_files(o["input"]):
            with open(fn) as f:
                for line in f:
                    tok = delim.split(line.rstrip("\n").rstrip("\r"))
                    if len(tok) <= max(rc, ic):
                        continue  # the reader skips short lines
                    by_item.setdefault(java_parse_long(tok[ic]), set()).add(java_parse_long(tok[rc]))
        items = np.array(sorted(by_item), np.int64)
        off = np.zeros(items.size + 1, np.int64)
        keys = []
        for r, it in enumerate(items):
            keys.extend(sorted(by_item[int(it)]))
            off[r + 1] = len(keys)
        outdir = os.path.join(o["output"], "similarity-matrix")
        os.makedirs(outdir, exist_ok=True)
        out = os.path.join(outdir, "part-00000")
        if items.size == 0:
            open(out, "w").close()
            return 0
        k = min(int(o["maxSimilaritiesPerItem"]), items.size)
        with _sketch_table(items, off, np.array(keys, np.int64), None, int(o["sketchDepth"]),
                           int(o["sketchWidth"]), int(o["hashSeed"]), device) as t:
            t.write_similarities(out, k, "spark_itemsimilarity")
        return 0


def main(argv=None):
    """python -m mahout_amd.jobs itemsimilarity|spark-itemsimilarity <options>"""
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("itemsimilarity", "spark-itemsimilarity"):
        print(main.__doc__)
        return 2
    job = ItemSimilarityJob() if argv[0] == "itemsimilarity" else ItemSimilarityDriver()
    try:
        return job.run(argv[1:])
    except _lib.CmsError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    raise SystemExit(main())

"""CPU: the Java drop-in classes respect the reference base classes' contract.

No JDK exists in the image, so integration/java is not compiled here.  This
test catches the class of error a ctypes replay cannot: a replacement class
overriding a method its base class declares `final` (javac rejects it) or
missing an abstract one.  The base classes' final / abstract methods come from
a committed fixture (tests/golden/java_final_methods.json, generated from
`T/impl/similarity/AbstractSimilarity.java` and `AbstractItemSimilarity.java`
by tests/golden/make_java_finals.py), so the reference is not read here.
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "integration", "java", "org", "apache", "mahout", "cf", "taste", "impl", "similarity")
FIXTURE = os.path.join(ROOT, "tests", "golden", "java_final_methods.json")

MODS = {"public", "protected", "private", "final", "abstract", "static", "synchronized", "native"}
DECL = re.compile(r"^  ((?:\w+\s+)*)([\w<>\[\]]+)\s+(\w+)\s*\(([^)]*)\)")


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _members(path):
    """Top-level member methods of the public class (two-space indent):
    (name, [param types], modifiers)."""
    out = []
    for line in _strip_comments(open(path).read()).splitlines():
        m = DECL.match(line)
        if not m:
            continue
        mods = set(m.group(1).split())
        if not mods <= MODS:
            continue
        params = []
        for p in [x.strip() for x in m.group(4).split(",") if x.strip()]:
            params.append(re.sub(r"\bfinal\s+", "", p).rsplit(None, 1)[0])
        out.append((m.group(3), params, mods))
    return out


def _extends(path):
    m = re.search(r"\bclass\s+\w+\s+extends\s+(\w+)", _strip_comments(open(path).read()))
    return m.group(1) if m else None


def _chain(fx, cls):
    while cls:
        yield cls, fx["classes"][cls]
        cls = fx["classes"][cls]["extends"]


def test_fixture_lists_the_reference_finals():
    fx = json.load(open(FIXTURE))
    finals = {(m["name"], tuple(m["params"])) for m in fx["classes"]["AbstractSimilarity"]["final_methods"]}
    assert ("refresh", ("Collection<Refreshable>",)) in finals  # AbstractSimilarity.java:333
    assert ("toString", ()) in finals  # AbstractSimilarity.java:339


def test_dropins_override_no_final_method_and_implement_abstract_ones():
    fx = json.load(open(FIXTURE))
    checked = 0
    for fname in sorted(os.listdir(JAVA)):
        if not fname.endswith(".java"):
            continue
        path = os.path.join(JAVA, fname)
        parent = _extends(path)
        if parent not in fx["classes"]:
            continue
        own = {(name, tuple(params)) for name, params, mods in _members(path) if "static" not in mods}
        for cls, spec in _chain(fx, parent):
            for m in spec["final_methods"]:
                sig = (m["name"], tuple(m["params"]))
                assert sig not in own, f"{fname} overrides final {cls}.{m['name']} ({cls}.java:{m['line']})"
        for cls, spec in _chain(fx, parent):
            for m in spec["abstract_methods"]:
                sig = (m["name"], tuple(m["params"]))
                assert sig in own, f"{fname} does not implement abstract {cls}.{m['name']}"
        checked += 1
    assert checked >= 2  # CosineCM (extends AbstractSimilarity) and CosineCMGpu (AbstractItemSimilarity)


def test_cosinecm_refresh_semantics_documented():
    src = open(os.path.join(JAVA, "CosineCM.java")).read()
    assert "ensureCurrent()" in src and "public void rebuild()" in src
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "never clears" in integ  # the reference's sketches cache (CosineCM.java:60-67)


def test_native_calls_hold_the_handle_lock():
    """a lazy rebuild may swap and destroy the handle while other
    threads query.  Every native call on the handle must run between
    acquire() (read side of the handle lock) and release(); only build()'s
    swap and close() destroy a handle, under the write side."""
    src = _strip_comments(open(os.path.join(JAVA, "CosineCMGpu.java")).read())
    body = src[src.index("class CosineCMGpu"):src.index("private static native")]  # up to the JNI declarations
    calls = re.findall(r"\bnative(?!Create|Destroy|SetHashParams|SetOwnerIds|IngestCsr|SetOwnerDeltaEpsilon|"
                       r"ConfigureOwnerShapes|Finalize)\w+\((\w+)", body)
    assert calls and all(c == "h" for c in calls), calls
    # each `long h = acquire();` is followed by a try/finally release(), and
    # every native call on the handle lies inside one of those spans
    spans = []
    for m in re.finditer(r"long h = acquire\(\);\s*try \{(.*?)\} finally \{\s*release\(\);", body, re.S):
        assert "native" in m.group(1)
        spans.append((m.start(1), m.end(1)))
    assert body.count("long h = acquire();") == body.count("release();") - 0
    call_pos = [m.start() for m in re.finditer(r"\bnative(?!Create|Destroy|SetHashParams|SetOwnerIds|IngestCsr|"
                                               r"SetOwnerDeltaEpsilon|ConfigureOwnerShapes|Finalize)\w+\(h\b", body)]
    assert len(call_pos) == len(calls)
    assert all(any(a <= c < b for a, b in spans) for c in call_pos)
    destroy = [m.start() for m in re.finditer(r"nativeDestroy\(", body)]
    wl = [m.start() for m in re.finditer(r"writeLock\(\)\.lock\(\)", body)]
    # every destroy of a live (published) handle sits after a write-lock
    # acquisition; the one in build()'s error path destroys an unpublished one
    assert len(wl) >= 2 and sum(1 for d in destroy if any(w < d for w in wl)) >= 2

"""Generate tests/golden/java_final_methods.json from the reference's Taste
base classes (run in the build container, where /root/reference exists).

The fixture is data: for each base class the replacement classes extend
(`T/impl/similarity/AbstractSimilarity.java`, `AbstractItemSimilarity.java`),
the methods declared `final` (a subclass may not override them) and
`abstract` (a subclass must implement them), as name + parameter types.
tests/test_java_dropin.py checks integration/java against it without
touching the reference.

    python tests/golden/make_java_finals.py
"""
import json
import os
import re

REF = "/root/reference/mr/src/main/java/org/apache/mahout/cf/taste/impl/similarity"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "java_final_methods.json")

MODS = {"public", "protected", "private", "final", "abstract", "static", "synchronized"}
# a member declaration: two-space indent, modifiers, return type, name, parameters
DECL = re.compile(r"^  ((?:\w+\s+)*)([\w<>\[\]]+)\s+(\w+)\s*\(([^)]*)\)")


def param_types(params):
    out = []
    for p in [x.strip() for x in params.split(",") if x.strip()]:
        p = re.sub(r"\bfinal\s+", "", p)
        out.append(p.rsplit(None, 1)[0])
    return out


def scan(path):
    finals, abstracts = [], []
    for ln, line in enumerate(open(path), 1):
        m = DECL.match(line)
        if not m:
            continue
        mods = set(m.group(1).split())
        if not mods <= MODS:
            continue
        rec = {"name": m.group(3), "params": param_types(m.group(4)), "returns": m.group(2), "line": ln}
        if "final" in mods:
            finals.append(rec)
        if "abstract" in mods:
            abstracts.append(rec)
    return finals, abstracts


def main():
    out = {"source": "mr/src/main/java/org/apache/mahout/cf/taste/impl/similarity (jalhajj/mahout)", "classes": {}}
    for cls, parent in (("AbstractItemSimilarity", None), ("AbstractSimilarity", "AbstractItemSimilarity")):
        finals, abstracts = scan(os.path.join(REF, cls + ".java"))
        out["classes"][cls] = {"extends": parent, "final_methods": finals, "abstract_methods": abstracts}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()

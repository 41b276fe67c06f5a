"""INTEGRATION.md must not drift from the C-ABI (the
documented ecg_agg_update_parity had 8 arguments, the exported one 12).

Every call of a library function written in INTEGRATION.md -- in its tables,
its prose and its C examples -- must name a symbol the version script exports
(daos_amd/csrc/exports.map) and pass exactly as many arguments as that
function's prototype in include/*.h declares."""
import glob
import os
import re

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _exports():
    txt = open(os.path.join(ROOT, "daos_amd", "csrc", "exports.map")).read()
    glob_part = txt.split("global:")[1].split("local:")[0]
    return {s.strip().rstrip(";") for s in glob_part.split() if s.strip().rstrip(";")}


def _balanced(text, i):
    """text[i] == '(': the argument text up to the matching ')' (None if unbalanced)."""
    depth = 0
    for j in range(i, len(text)):
        if text[j] == "(":
            depth += 1
        elif text[j] == ")":
            depth -= 1
            if depth == 0:
                return text[i + 1:j]
    return None


def _nargs(args):
    args = re.sub(r"/\*.*?\*/", "", args, flags=re.S).strip()
    if args in ("", "void"):
        return 0
    depth, n = 0, 1
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            n += 1
    return n


def _prototypes():
    protos = {}
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(", txt):
            name = m.group(1)
            args = _balanced(txt, m.end() - 1)
            if args is None:
                continue
            rest = txt[m.end() + len(args):m.end() + len(args) + 3]
            # a declaration: "name(...);" preceded by a return type on the same statement
            if rest.startswith(");") and name not in protos:
                protos[name] = _nargs(args)
    return protos


def _doc_calls(exports):
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    calls = []
    for m in re.finditer(r"\b([A-Za-z_]\w*)\(", txt):
        if m.group(1) not in exports:
            continue
        args = _balanced(txt, m.end() - 1)
        if args is None or "..." in args or "\n\n" in args:
            continue
        calls.append((m.group(1), _nargs(args), txt[:m.start()].count("\n") + 1))
    return calls


def test_integration_calls_match_exports_and_prototypes():
    exports = _exports()
    protos = _prototypes()
    missing = sorted(n for n in exports if n not in protos)
    assert not missing, f"exported but no prototype found in include/*.h: {missing}"
    calls = _doc_calls(exports)
    assert len(calls) >= 25, calls          # the document really names the API
    bad = [(n, got, protos[n], line) for n, got, line in calls if got != protos[n]]
    assert not bad, "INTEGRATION.md argument counts differ from include/*.h: " + ", ".join(
        f"{n} line {line}: {got} args, prototype has {want}" for n, got, want, line in bad)


def test_integration_names_only_exported_functions():
    """Every ecg_* / ISA-L-looking identifier followed by '(' in the document is
    an exported function (no renamed or removed entry point lingers)."""
    exports = _exports()
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    names = set(re.findall(r"\b(ecg_\w+)\(", txt))
    assert names, "no ecg_ calls found"
    assert not sorted(names - exports), sorted(names - exports)

"""The Go plugin (application/grep_gpu.go) builds as INTEGRATION.md documents.

There is no Go toolchain here or on the GPU box, so these tests restate the two
rules of `go build` that decide whether the plugin compiles next to the
reference's application/grep.go:

* build constraints (`//go:build expr` before the package clause) choose the
  files of a package build; files named on the command line are all taken
  (go's `UseAllFiles` for command-line files);
* a package may declare each top-level name once ("Map redeclared in this
  block" otherwise).

For every documented command the files the build would take must declare
disjoint top-level names and export Map / Reduce with the reference's
signatures (application/grep.go:13,38; looked up by main/worker_launch.go:21-34).
CPU only; the reference's grep.go is read when present (this container), and
its declarations are pinned below for machines without it.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPU_GO = os.path.join(ROOT, "application", "grep_gpu.go")
REF_GO = "/root/reference/application/grep.go"
# The reference's application/grep.go as declarations (grep.go:11,13,38),
# used when the reference tree is absent.
REF_DECLS = {
    "pattern": "var",
    "Map": "func(filename string, contents string) []mapreduce.KeyValue",
    "Reduce": "func(key string, values []string) string",
}
# the line INTEGRATION.md asks a maintainer to add at the top of grep.go
REF_PATCH = "//go:build !dgrep_gpu"
HOST_TAGS = {"linux", "amd64", "cgo", "gc", "unix", "go1.18"}


def strip_go(src):
    """Source with comments and string/rune literals blanked (newlines kept)."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("".join(ch if ch == "\n" else " " for ch in src[i:j]))
            i = j
        elif c in "\"'`":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if (src[j] == "\\" and c != "`") else 1
            out.append(c + " " * (j - i - 1) + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def build_constraint(src):
    """The file's //go:build expression (None: no constraint). Only blank lines
    and line comments may precede it, and it must come before the package clause."""
    for line in src.splitlines():
        s = line.strip()
        if s.startswith("//go:build "):
            return s[len("//go:build "):].strip()
        if s == "" or s.startswith("//"):
            continue
        return None
    return None


def eval_constraint(expr, tags):
    """Evaluate a //go:build expression (identifiers, !, &&, ||, parentheses)."""
    toks = re.findall(r"\(|\)|!|&&|\|\||[A-Za-z0-9_.]+", expr)
    pos = [0]

    def peek():
        return toks[pos[0]] if pos[0] < len(toks) else None

    def take():
        pos[0] += 1
        return toks[pos[0] - 1]

    def atom():
        t = take()
        if t == "!":
            return not atom()
        if t == "(":
            v = orx()
            assert take() == ")"
            return v
        return t in tags

    def andx():
        v = atom()
        while peek() == "&&":
            take()
            v = atom() and v
        return v

    def orx():
        v = andx()
        while peek() == "||":
            take()
            v = andx() or v
        return v

    v = orx()
    assert pos[0] == len(toks), "bad //go:build expression: %r" % expr
    return v


def top_level_decls(src):
    """{name: declaration} of the package-level names a Go file declares
    (func without receiver, var, const, type; grouped forms included)."""
    s = strip_go(src)
    decls = {}
    depth = 0
    i, n = 0, len(s)
    group = None  # keyword of an open `var ( ... )` group at depth 1
    line_start = True
    while i < n:
        c = s[i]
        if c in "({[":
            depth += 1
            i += 1
            continue
        if c in ")}]":
            depth -= 1
            if depth == 0:
                group = None
            i += 1
            continue
        if depth == 0 or (depth == 1 and group):
            m = re.compile(r"(func|var|const|type)\b\s*").match(s, i) if depth == 0 else None
            if m:
                kw = m.group(1)
                j = m.end()
                if kw == "func":
                    if s[j] == "(":  # method: not a package-level name
                        i = j
                        continue
                    fm = re.compile(r"([A-Za-z_]\w*)\s*(\([^)]*\))\s*([^{\n]*)").match(s, j)
                    sig = re.sub(r"\s+", " ", "func" + fm.group(2) + " " + fm.group(3)).strip()
                    decls.setdefault(fm.group(1), []).append(sig)
                    i = fm.end()
                    continue
                if s[j] == "(":
                    group = kw
                    i = j
                    continue
                nm = re.compile(r"[A-Za-z_]\w*").match(s, j)
                decls.setdefault(nm.group(0), []).append(kw)
                i = nm.end()
                continue
            if depth == 1 and group and line_start:
                nm = re.compile(r"[ \t]*([A-Za-z_]\w*)").match(s, i)
                if nm:
                    decls.setdefault(nm.group(1), []).append(group)
                    i = nm.end()
                    line_start = False
                    continue
        line_start = c == "\n"
        i += 1
    return decls


def reference_source(patched):
    if os.path.exists(REF_GO):
        src = open(REF_GO).read()
    else:
        src = "package main\n\n" + "".join(
            ("var %s string = \"\"\n" % k) if v == "var" else "func %s%s { }\n" % (k, v[4:])
            for k, v in REF_DECLS.items())
    return (REF_PATCH + "\n\n" + src) if patched else src


def files_of_build(cmd_files, tags, patched):
    """Files (name -> source) a documented `go build` takes: `cmd_files` named on
    the command line (all taken), or None for the package ./application, whose
    files are filtered by their constraints."""
    pkg = {"grep.go": reference_source(patched), "grep_gpu.go": open(GPU_GO).read()}
    if cmd_files is not None:
        return {f: pkg[f] for f in cmd_files}
    out = {}
    for name, src in pkg.items():
        expr = build_constraint(src)
        if expr is None or eval_constraint(expr, tags | HOST_TAGS):
            out[name] = src
    return out


def collisions(files):
    seen, dup = {}, []
    for name, src in files.items():
        for d in top_level_decls(src):
            if d in ("init", "_"):  # may be declared any number of times
                continue
            if d in seen:
                dup.append((d, seen[d], name))
            seen[d] = name
    return dup


def test_constraint_evaluator():
    assert eval_constraint("dgrep_gpu", {"dgrep_gpu"})
    assert not eval_constraint("!dgrep_gpu", {"dgrep_gpu"})
    assert eval_constraint("linux && (amd64 || arm64) && !dgrep_gpu", {"linux", "amd64"})
    assert not eval_constraint("linux && !(amd64 || arm64)", {"linux", "amd64"})


def test_decl_parser_sees_both_files():
    ref = top_level_decls(reference_source(False))
    assert set(ref) == set(REF_DECLS)
    gpu = top_level_decls(open(GPU_GO).read())
    # grep_gpu.go: the three reference names plus its own helpers
    assert {"pattern", "Map", "Reduce"} <= set(gpu)
    assert all(len(v) == 1 for v in gpu.values()), gpu
    # a file that redeclares is caught
    assert collisions({"a.go": "package main\nfunc Map() {}\n", "b.go": "package main\nvar (\n\tx int\n\tMap int\n)\n"})


@pytest.mark.skipif(not os.path.exists(REF_GO), reason="reference tree absent")
def test_pinned_reference_declarations():
    ref = top_level_decls(open(REF_GO).read())
    assert {k: v[0] for k, v in ref.items()} == {"pattern": "var", "Map": REF_DECLS["Map"],
                                                 "Reduce": REF_DECLS["Reduce"]}


def test_plugin_file_has_constraint_and_no_paths():
    src = open(GPU_GO).read()
    assert build_constraint(src) == "dgrep_gpu"
    # the constraint is followed by a blank line (else it is package documentation)
    lines = src.splitlines()
    k = next(i for i, l in enumerate(lines) if l.startswith("//go:build"))
    assert lines[k + 1].strip() == ""
    cgo = [l for l in src.splitlines() if l.strip().startswith("#cgo")]
    assert cgo and all("${SRCDIR}" not in l and "-I" not in l and "-L" not in l for l in cgo), cgo


@pytest.mark.parametrize("cmd_files,tags,patched", [
    (["grep_gpu.go"], set(), False),          # (a) go build ./application/grep_gpu.go
    (None, {"dgrep_gpu"}, True),              # (b) go build -tags dgrep_gpu ./application
    (None, set(), True),                      # the package without the tag: the reference plugin as before
    (None, set(), False),                     # the reference tree with grep_gpu.go copied in, untagged
])
def test_documented_builds_compile_one_map(cmd_files, tags, patched):
    files = files_of_build(cmd_files, tags, patched)
    assert not collisions(files), collisions(files)
    decls = {}
    for src in files.values():
        decls.update({k: v[0] for k, v in top_level_decls(src).items()})
    # exactly one Map / Reduce with the plugin signatures worker_launch.go asserts
    assert decls["Map"] == REF_DECLS["Map"]
    assert decls["Reduce"] == REF_DECLS["Reduce"]
    want_gpu = cmd_files is not None or "dgrep_gpu" in tags
    assert ("grep_gpu.go" in files) == want_gpu


def test_unconstrained_package_build_would_collide():
    """Why the constraint is needed: both files in one package build redeclare."""
    files = {"grep.go": reference_source(False), "grep_gpu.go": open(GPU_GO).read()}
    names = {d for d, _, _ in collisions(files)}
    assert {"pattern", "Map", "Reduce"} <= names


def test_integration_documents_the_commands():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert REF_PATCH in doc
    assert "go build -buildmode=plugin -o grep.so ./application/grep_gpu.go" in doc
    assert "go build -tags dgrep_gpu -buildmode=plugin -o grep.so ./application" in doc
    assert "go build -buildmode=plugin -o grep.so ./application\n" not in doc

"""INTEGRATION.md section 2's Rust `extern "C"` block against include/rsvio_gpu.h (verdict r04
item 4): the block a maintainer pastes into the reference crate (whose toolchain, cargo/rustc, is
absent here) declares EVERY exported entry point with the header's parameter count, and each
parameter's kind (pointer vs scalar, const vs mut pointee, scalar width) agrees.  The Rust text is
parsed on its own, not through tools/gen_rust_ffi.py, so a hand edit of either side is caught."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "rsvio_gpu.h"
DOC = ROOT / "INTEGRATION.md"

# parity-only / diagnostic entry points a Rust caller never needs; none are exempt today (the
# block carries all of them), the list is where a future exemption would be stated explicitly
EXEMPT: set[str] = set()


def header_protos():
    text = re.sub(r"/\*.*?\*/", " ", HEADER.read_text(), flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    out = {}
    for m in re.finditer(r"(?m)^\s*((?:const\s+)?\w+\s*\**)\s*\b(rsvio_\w+)\s*\(([^;{]*?)\)\s*;", text):
        args = " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        out[m.group(2)] = (m.group(1).strip(), params)
    return out


def rust_protos():
    doc = DOC.read_text()
    i = doc.index('extern "C" {')
    body = doc[i:doc.index("\n}\n", i)]
    body = re.sub(r"//[^\n]*", " ", body)
    out = {}
    for m in re.finditer(r"pub fn (rsvio_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", body, re.S):
        args = " ".join(m.group(2).split())
        params = [] if not args else [a.split(":", 1)[1].strip() for a in args.split(",")]
        out[m.group(1)] = ((m.group(3) or "()").strip(), params)
    return out


C_SCALAR = {"int": "c_int", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "size_t": "usize",
            "double": "f64", "float": "f32", "uint8_t": "u8", "char": "c_char", "void": "c_void"}


def c_kind(decl):
    """('ptr', [const per level, innermost first], base) or ('val', base) of a C parameter/return."""
    toks = decl.replace("*", " * ").split()
    if len(toks) > 1 and toks[-1] not in ("*", "const"):
        toks = toks[:-1]                       # the parameter's name
    const = toks[0] == "const"
    toks = toks[1:] if const else toks
    base, levels, cur = toks[0], [], const
    for t in toks[1:]:
        if t == "*":
            levels.append(cur)
            cur = False
        elif t == "const":
            cur = True
    base = C_SCALAR.get(base, base)
    return ("ptr", levels, base) if levels else ("val", base)


def rust_kind(t):
    levels = []
    t = t.strip()
    while t.startswith("*"):
        m = re.match(r"\*(const|mut)\s+(.*)", t)
        levels.append(m.group(1) == "const")
        t = m.group(2).strip()
    return ("ptr", levels[::-1], t) if levels else ("val", t)


def test_block_declares_every_header_entry_point():
    h, r = header_protos(), rust_protos()
    assert len(h) >= 67
    missing = sorted(set(h) - set(r) - EXEMPT)
    extra = sorted(set(r) - set(h))
    assert not missing, f"INTEGRATION.md lacks {missing} (run tools/gen_rust_ffi.py --write)"
    assert not extra, f"INTEGRATION.md declares {extra}, absent from the header"


def test_parameter_counts_and_kinds_match():
    h, r = header_protos(), rust_protos()
    for name, (ret, params) in h.items():
        if name in EXEMPT:
            continue
        rret, rparams = r[name]
        assert len(rparams) == len(params), (name, params, rparams)
        for c, rs in zip(params, rparams):
            assert c_kind(c) == rust_kind(rs), (name, c, rs)
        if ret == "void":
            assert rret == "()", name
        else:
            assert c_kind(ret + " x") == rust_kind(rret), (name, ret, rret)


def test_documented_modes_are_declared():
    """The pipelined and look-ahead modes INTEGRATION section 3 tells a Rust caller to use."""
    r = rust_protos()
    for s in ("rsvio_ba_set_stream", "rsvio_pnp_set_stream", "rsvio_tracker_submit_device", "rsvio_ba_run",
              "rsvio_ba_batch_create", "rsvio_ba_batch_run", "rsvio_ba_batch_destroy", "rsvio_unproject_d",
              "rsvio_tracker_submit", "rsvio_tracker_collect", "rsvio_ba_run_async", "rsvio_ba_wait"):
        assert s in r, s

"""Generate the Rust `extern "C"` block of INTEGRATION.md section 2 from include/rsvio_gpu.h.

Every prototype of the header becomes one `pub fn` with the same name and parameters (C types
mapped to their Rust FFI equivalents); the comment line above a group in the header is carried
over.  tests/test_rust_ffi_cpu.py checks the block in INTEGRATION.md against the header, so a
header change without a regenerated block fails on CPU.

usage: python tools/gen_rust_ffi.py            # prints the block
       python tools/gen_rust_ffi.py --write    # replaces the block in INTEGRATION.md
"""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "rsvio_gpu.h"
DOC = ROOT / "INTEGRATION.md"
BEGIN, END = "extern \"C\" {\n", "\n}\n"

SCALAR = {"int": "c_int", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "size_t": "usize",
          "double": "f64", "float": "f32", "uint8_t": "u8", "char": "c_char", "void": "c_void"}


def prototypes(text=None):
    """[(return C type, name, [(param C type, param name)])] in header order."""
    text = text if text is not None else HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    out = []
    for m in re.finditer(r"(?m)^\s*((?:const\s+)?[\w]+\s*\**)\s*\b(rsvio_\w+)\s*\(([^;{]*?)\)\s*;", text):
        ret, name, args = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                pm = re.match(r"(.*?)(\w+)$", a)
                params.append((pm.group(1).strip(), pm.group(2)))
        out.append((ret, name, params))
    return out


def rust_type(c):
    c = " ".join(c.replace("*", " * ").split())
    toks = c.split()
    # pointer levels, innermost first: "const T * const *" -> T, [const, const]
    base_const = toks[0] == "const"
    if base_const:
        toks = toks[1:]
    base = toks[0]
    rest = toks[1:]
    levels = []  # constness of each pointee level, innermost first
    cur_const = base_const
    for t in rest:
        if t == "*":
            levels.append(cur_const)
            cur_const = False
        elif t == "const":
            cur_const = True
    r = SCALAR.get(base, base)
    for is_const in levels:
        r = ("*const " if is_const else "*mut ") + r
    return r


def snake(name):
    return {"R": "r", "T_W_B": "t_w_b", "p_W": "p_w"}.get(name, name.lower())


GROUPS = {
    "rsvio_last_error": "errors, device query, CU-masked streams",
    "rsvio_tracker_create": "StereoPatchTracker (feature_tracker.rs:91-206); submit / collect = the one-frame look-ahead",
    "rsvio_pyramid_bytes": "parity entry points: build_image_pyramid (:209-220), track_points (:252-291), "
                           "detect_key_points (image_utilities.rs:108-175)",
    "rsvio_track_ctx_create": "batched serving: many track_points batches per launch (device pointers)",
    "rsvio_ft_create": "feature_tracker/ crate: FeatureTracker (feature_tracker/src/feature_tracker.rs:51-194) "
                       "and its parity entry points",
    "rsvio_sincosf": "the glibc sinf / cosf restatement (parity diagnostics)",
    "rsvio_unproject": "Frame::add_*_feature unprojection (frame.rs:107-134)",
    "rsvio_ba_create": "SlidingWindow::optimize's solver (sliding_window.rs:159-381 + apex LM); set_problem + "
                       "run_async + wait = the pipelined estimator",
    "rsvio_ba_batch_create": "batched BA: many independent windows per launch chain",
    "rsvio_rccl_unique_id": "landmark-sharded BA (DESIGN.md section 8): RCCL, then the P2P one-shot exchange",
    "rsvio_pnp_create": "SlidingWindow::track_motion + keyframe rule (sliding_window.rs:490-587, estimator.rs:195-234)",
    "rsvio_quat_from_matrix": "host-only: UnitQuaternion::from_matrix (:221), window build / apply (:174-300, :418-486)",
    "rsvio_pnp_set_stream": "motion tracking (continued)",
}


def wrap(head, parts, tail, width=112):
    """`head(p1, p2, ...)tail`, continued lines indented by 8 when longer than width."""
    lines, cur = [], "    " + head + "("
    for i, p in enumerate(parts):
        piece = p + (", " if i + 1 < len(parts) else "")
        if len(cur) + len(piece.rstrip()) > width and cur.strip():
            lines.append(cur.rstrip())
            cur = "        "
        cur += piece
    lines.append(cur + ")" + tail)
    return lines


def block():
    lines = []
    for ret, name, params in prototypes():
        if name in GROUPS:
            lines.append(f"    // {GROUPS[name]}")
        rt = "" if ret == "void" else f" -> {rust_type(ret)}"
        lines += wrap(f"pub fn {name}", [f"{snake(n)}: {rust_type(t)}" for t, n in params], rt + ";")
    return BEGIN + "\n".join(lines) + END


def main():
    b = block()
    if "--write" not in sys.argv:
        print(b)
        return
    doc = DOC.read_text()
    i = doc.index(BEGIN)
    j = doc.index(END, i) + len(END)
    DOC.write_text(doc[:i] + b + doc[j:])


if __name__ == "__main__":
    main()

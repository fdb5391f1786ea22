"""Scan the gfx950 ISA of the HIP kernels for the compiler-made serial stalls
that the round-6 attention / stem fixes removed (docs/benchmarks.md, "BERT
attention: staging ..." and "ResNet stem: ..."):

  * wait-before-store: a load issued inside an exec-masked block and waited for
    on the spot (``s_and_saveexec`` ... load ... ``s_waitcnt vmcnt(0)`` before
    the block closes) -- a guarded load the compiler sank into its branch, one
    serial memory round trip each;
  * lds-serial: ``ds_read`` -> ``s_waitcnt lgkmcnt(0)`` -> MFMA with no other
    read in flight -- each MFMA group waits a full LDS round trip;
  * vmcnt0-in-loop: ``s_waitcnt vmcnt(0)`` inside a loop body (drains every
    load, store and LDS-DMA of the wave, prefetches included);
  * int-bf16: the integer round-to-nearest bf16 sequence (``v_bfe_u32 ... 16, 1``
    + ``v_add3_u32 ... 0x7fff``) instead of ``v_cvt_pk_bf16_f32``.

Counts are per kernel symbol; a count is a place to look, not a verdict (a
2-stage ring's loop is meant to drain vmcnt, an epilogue's guarded store may be
fine).  CPU only: hipcc -S --cuda-device-only.

    python scripts/isa_audit.py                       # every kernels/*.hip
    python scripts/isa_audit.py attention.hip stem.hip --kernel attention_kernel
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "rust_tensorflow_serving2_amd", "kernels")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

LOAD = re.compile(r"^\s*(global_load|buffer_load|flat_load)\w*\s+v")
MFMA = re.compile(r"^\s*v_mfma_")
DSREAD = re.compile(r"^\s*ds_read")
WAIT_VM0 = re.compile(r"^\s*s_waitcnt\s+vmcnt\(0\)")
WAIT_LGKM0 = re.compile(r"^\s*s_waitcnt\s+lgkmcnt\(0\)\s*$")
LABEL = re.compile(r"^(\.LBB\w+):")
BRANCH = re.compile(r"^\s*s_cbranch_\w+\s+(\.LBB\w+)")
SAVEEXEC = re.compile(r"^\s*s_and_saveexec_b64")
RESTORE = re.compile(r"^\s*s_or_b64\s+exec,\s*exec")


def compile_asm(src: str) -> str:
    out = tempfile.NamedTemporaryFile(suffix=".s", delete=False).name
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-gpu-rdc", "--cuda-device-only", "-S",
           "-o", out, src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        raise SystemExit(f"hipcc failed on {src}")
    with open(out) as f:
        text = f.read()
    os.unlink(out)
    return text


def kernels(asm: str):
    """(symbol, lines) of every kernel body (symbol label .. s_endpgm)."""
    lines = asm.splitlines()
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\w+):", lines[i])
        if m:
            j = i + 1
            while j < len(lines) and "s_endpgm" not in lines[j]:
                j += 1
            yield m.group(1), lines[i + 1:j + 1]
            i = j
        i += 1


def demangle(sym: str) -> str:
    try:
        return subprocess.run(["c++filt", sym], capture_output=True, text=True).stdout.strip() or sym
    except OSError:
        return sym


def audit(body):
    code = [ln for ln in body if ln.strip() and not ln.lstrip().startswith(";")]
    label_at = {}
    for idx, ln in enumerate(code):
        m = LABEL.match(ln)
        if m:
            label_at[m.group(1)] = idx
    # loop bodies: a backward branch from idx to an earlier label
    loops = []
    for idx, ln in enumerate(code):
        m = BRANCH.match(ln)
        if m and m.group(1) in label_at and label_at[m.group(1)] < idx:
            loops.append((label_at[m.group(1)], idx))
    in_loop = [False] * len(code)
    for a, b in loops:
        for k in range(a, b + 1):
            in_loop[k] = True
    res = {"wait-before-store": 0, "lds-serial": 0, "vmcnt0-in-loop": 0, "int-bf16": 0}
    masked, pending_load = False, False
    for idx, ln in enumerate(code):
        if SAVEEXEC.match(ln):
            masked, pending_load = True, False
        elif RESTORE.match(ln):
            masked, pending_load = False, False
        elif masked and LOAD.match(ln):
            pending_load = True
        elif masked and pending_load and WAIT_VM0.match(ln):
            res["wait-before-store"] += 1
            pending_load = False
        if WAIT_VM0.match(ln) and in_loop[idx]:
            res["vmcnt0-in-loop"] += 1
        if WAIT_LGKM0.match(ln) and idx + 1 < len(code) and MFMA.match(code[idx + 1]):
            # the read it waits for is the only one in flight: no other ds_read
            # between the previous MFMA and this wait
            k, reads = idx - 1, 0
            while k >= 0 and not MFMA.match(code[k]) and not LABEL.match(code[k]):
                reads += bool(DSREAD.match(code[k]))
                k -= 1
            if reads == 1:
                res["lds-serial"] += 1
        if "v_bfe_u32" in ln and re.search(r",\s*16,\s*1\s*$", ln):
            nxt = " ".join(code[idx + 1:idx + 3])
            if "v_add3_u32" in nxt:
                res["int-bf16"] += 1
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*", help="kernel sources (default: every kernels/*.hip)")
    ap.add_argument("--kernel", default="", help="only symbols whose demangled name contains this")
    ap.add_argument("--all", action="store_true", help="also list kernels with no findings")
    a = ap.parse_args()
    files = [f if os.path.isabs(f) else os.path.join(KDIR, f) for f in a.files] or sorted(glob.glob(f"{KDIR}/*.hip"))
    for src in files:
        asm = compile_asm(src)
        for sym, body in kernels(asm):
            name = demangle(sym)
            if a.kernel and a.kernel not in name:
                continue
            r = audit(body)
            if a.all or any(r.values()):
                flags = "  ".join(f"{k}={v}" for k, v in r.items() if v or a.all)
                print(f"{os.path.basename(src):14s} {name[:90]:90s} {flags}")


if __name__ == "__main__":
    main()

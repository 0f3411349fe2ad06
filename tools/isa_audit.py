"""ISA audit of one kernel: compiles a csrc/*.hip file to gfx950 assembly and
prints the kernel's register/scratch budget and counts of instructions worth
knowing about (scratch, flat, readlane, MFMA, s_cbranch) in its body.

  python tools/isa_audit.py topk_f16.hip flatip_topk_v4_scan [-D NAME ...]
"""
import argparse
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(__file__), "..", "real-time-recommendation-system-with-feature-store_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("-o", default="/tmp/audit.s")
    ap.add_argument("--nth", type=int, default=0, help="which matching kernel")
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-munsafe-fp-atomics", "-I" + os.path.join(CSRC, "..", "..", "include"), "-I" + CSRC,
           os.path.join(CSRC, a.src), "-o", a.o] + ["-D" + d for d in a.D]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(1)
    text = open(a.o).read()
    starts = [m for m in re.finditer(r"^(_Z\S*" + re.escape(a.kernel) + r"\S*):", text, re.M)]
    if not starts:
        sys.exit("kernel not found")
    m = starts[a.nth]
    name = m.group(1)
    end = text.find(".Lfunc_end", m.end())
    body = text[m.end():end]
    tail = text[end:end + 4000]

    def meta_val(key):
        mm = re.search(r";\s*" + key + r":\s*(\d+)", tail)
        return mm.group(1) if mm else "?"

    print(name)
    for key in ("NumVgprs", "NumAgprs", "NumSgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
        print(f"  {key:28s} {meta_val(key)}")
    ins = [ln.strip().split()[0] for ln in body.splitlines() if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
    cnt = lambda pred: sum(1 for i in ins if pred(i))
    print(f"  instructions                 {len(ins)}")
    print(f"  mfma                         {cnt(lambda i: 'mfma' in i)}")
    print(f"  scratch ops                  {cnt(lambda i: i.startswith('scratch_') or i.startswith('buffer_store') or i.startswith('buffer_load'))}")
    print(f"  flat ops                     {cnt(lambda i: i.startswith('flat_'))}")
    print(f"  global_store                 {cnt(lambda i: i.startswith('global_store'))}")
    print(f"  v_readlane/writelane         {cnt(lambda i: i.startswith('v_readlane') or i.startswith('v_writelane'))}")
    print(f"  s_cbranch                    {cnt(lambda i: i.startswith('s_cbranch'))}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Diagnostics (not product): compile a csrc/*.hip file to gfx950 assembly and
report, per kernel, registers, spills, scratch instructions and the
instruction mix (tools/isa_stats.py [file.hip] [-D...])."""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd", "csrc")


def main():
    src = os.path.join(CSRC, "bb_env.hip")
    defs = []
    for a in sys.argv[1:]:
        if a.startswith("-D"):
            defs.append(a)
        else:
            src = a if os.path.isabs(a) else os.path.join(CSRC, a)
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    f"-I{os.path.join(REPO, 'include')}", "--cuda-device-only", "-S", *defs, "-o", out, src],
                   check=True, stderr=subprocess.DEVNULL)
    text = open(out).read().splitlines()
    kern = None
    body = collections.defaultdict(list)
    meta = {}
    for ln in text:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            kern = m.group(1)
            continue
        if ln.startswith("\t.size") or ln.startswith(".Lfunc_end"):
            kern = None
        if kern and re.match(r"^\s+[a-z]", ln) and not ln.strip().startswith("."):
            body[kern].append(ln.split()[0])
        m = re.match(r"^\s+\.set (_Z\S+)\.(num_vgpr|numbered_sgpr|private_seg_size), (\d+)", ln)
        if m:
            meta.setdefault(m.group(1), {})[m.group(2)] = int(m.group(3))
    for k, ins in body.items():
        name = re.sub(r"^_ZN2bb\d+", "", k)[:40]
        c = collections.Counter(ins)
        md = meta.get(k, {})
        print(f"{name:40s} vgpr {md.get('num_vgpr')} sgpr {md.get('numbered_sgpr')} scratch {md.get('private_seg_size')} "
              f"insts {len(ins)} valu {sum(v for x, v in c.items() if x.startswith('v_'))} "
              f"salu {sum(v for x, v in c.items() if x.startswith('s_'))} "
              f"scratch_ops {sum(v for x, v in c.items() if x.startswith('scratch_'))} "
              f"readlane {c['v_readlane_b32']} writelane {c['v_writelane_b32']}")


if __name__ == "__main__":
    main()

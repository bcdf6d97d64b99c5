"""ISA evidence for the forest walk (tools only): compiles csrc/fdx_forest.hip for gfx950 to
assembly, takes the default kernel (k_forest_rank<1024, 1, 10, 0, 102>), and prints

  * its register budget (VGPRs, scratch = spills, LDS, waves per SIMD),
  * for every basic block that holds walk steps (v_med3_i32 = one chain-step each): the
    instruction mix per chain-step and the s_waitcnt placement, and
  * the text of the steady-state block of the chunk size the bench runs most (6 trees:
    the one-group loop, 6 chains in 3 interleaved pairs, 4 unrolled steps per exit test).

usage: python3 tools/isa_excerpt.py [out.txt] [v2]
  v2: the rank-layout-v2 chunk-loop instantiation the deployed model runs
      (k_forest_rank<1024, 2, 2, 4, 2, true>: paired planes, one-tree chunks, two rows per lane)
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "real-time_fraud_detection_system_amd", "csrc")
KERNEL = "k_forest_rankILi1024ELi1ELi10ELi0ELi102ELb1E"  # the chunk-loop instantiation (large batches)


KERNEL_V2 = "k_forest_rankILi1024ELi2ELi2ELi4ELi2ELb1E"  # variant 5 (paired planes), the deployed default since r06


def kernel_body(asm):
    lines = asm.split("\n")
    start = next(i for i, l in enumerate(lines) if KERNEL in l and re.match(r"^_Z\S+:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    # the comment block right after the kernel carries its register / LDS summary
    summ, seen = [], set()
    for l in lines[end:]:
        m = re.match(r"\s*;\s*(NumVgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize|NumVGPRsForWavesPerEU)\b", l)
        if m:
            if m.group(1) in seen:
                break
            seen.add(m.group(1))
            summ.append(l.strip())
    return lines[start:end], summ


def blocks(body):
    out, cur, name = [], [], "entry"
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
        else:
            cur.append(l)
    out.append((name, cur))
    return out


def ops(block):
    r = []
    for l in block:
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        r.append(t.split(";")[0].strip())
    return r


def main():
    global KERNEL
    out = sys.argv[1] if len(sys.argv) > 1 else None
    v2 = len(sys.argv) > 2 and sys.argv[2] == "v2"
    if v2:
        KERNEL = KERNEL_V2
    asm_path = "/tmp/fdx_forest_isa.s"
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", asm_path,
                           os.path.join(CSRC, "fdx_forest.hip")])
    asm = open(asm_path).read()
    body, summ = kernel_body(asm)
    res = [("k_forest_rank<1024, 2, 2, 4, 2, true> (variant 5, rank layout v2 over paired planes: the deployed model; chunk loop)" if v2 else
            "k_forest_rank<1024, 1, 10, 0, 102, true> (default variant 1, chunk loop)") + ", gfx950, hipcc -O3",
           "register summary:"]
    res += ["  " + s for s in summ]
    res.append("")
    res.append("walk blocks (one v_med3_i32 per chain-step): per chain-step instruction counts")
    res.append(f"{'block':>14} {'steps':>5} {'ds_read':>7} {'VALU':>5} {'SALU':>5} {'waitcnt':>7} {'lgkm waits':<40}")
    walk = []
    for name, b in blocks(body):
        o = ops(b)
        n = sum(1 for x in o if x.startswith("v_med3_i32"))
        if n < (1 if v2 else 4):
            continue
        c = collections.Counter(x.split()[0] for x in o)
        ds = sum(v for k, v in c.items() if k.startswith("ds_read"))
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_nop", "s_cbranch",
                                                                                         "s_branch")))
        waits = [x for x in o if x.startswith("s_waitcnt")]
        lg = collections.Counter(re.sub(r"\s+", " ", w.split(None, 1)[1]) for w in waits)
        walk.append((name, n, o))
        res.append(f"{name:>14} {n:5d} {ds / n:7.2f} {valu / n:5.2f} {salu / n:5.2f} {len(waits) / n:7.2f} "
                   + ", ".join(f"{k} x{v}" for k, v in sorted(lg.items())))
    # the 6-chain steady-state interval: 24 med3 (6 chains x 4 steps)
    six = [w for w in walk if w[1] == (4 if v2 else 24)]
    if six:
        name, n, o = six[0]
        res += ["", f"steady-state interval ({name}: " + ("1 chain x 4 steps" if v2 else "6 chains x 4 steps")
                + "), in issue order:"]
        res += ["  " + x for x in o]
    text = "\n".join(res) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()

"""Static ISA account of the stream executor's phases (exe_local inlined in entry_exe<LW=true>):
the DGP_TRACE=3 build's s_memtime probes split the function's assembly into the phases
tools/link_profile.py measures; per phase, the instructions by class and the s_waitcnt that
wait for LDS (lgkmcnt) or memory (vmcnt) results.

    hipcc ... -DDGP_TRACE=3 --cuda-device-only -S dgplace.hip -o tr3.s
    python tools/isa_phases.py tr3.s [link_profile output]"""
import re
import sys

asm = open(sys.argv[1]).read().splitlines()
fn = "_ZN3dgp2st9entry_exeILb1EEEvv:"
a = next(i for i, l in enumerate(asm) if l.startswith(fn))
b = next(i for i in range(a + 1, len(asm)) if re.match(r"^_Z\w+:", asm[i]))
body = asm[a:b]
# trace slot k of a probe = the byte offset / 8 of the store that follows its s_memtime
SLOT = {2: "claim", 8: "precheck", 9: "state", 10: "compl_needs", 11: "pre_wait", 12: "post_wait",
        13: "keys", 14: "argmin_early", 15: "commit1", 16: "frontier", 17: "refill", 18: "w_release"}
marks = []
for i, l in enumerate(body):
    if "s_memtime" in l:
        for j in range(i + 1, min(i + 60, len(body))):
            m = re.search(r"(global|flat)_store_dwordx2 .*offset:(\d+)", body[j])
            if m:
                k = int(m.group(2)) // 8
                if k in SLOT and all(k != kk for _, kk in marks):
                    marks.append((i, k))
                break
order = [2, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18]
pos = {k: i for i, k in marks}
measured = {}
if len(sys.argv) > 2:
    for l in open(sys.argv[2]):
        m = re.match(r"\s+(\w+) -> (\w+)\s+mean\s+(\d+)", l)
        if m:
            measured[m.group(1)] = int(m.group(3))


def classify(lines):
    c = dict(total=0, valu=0, salu=0, lds=0, vmem=0, smem=0, branch=0, wait_lgkm=0, wait_vm=0)
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c["total"] += 1
        if op == "s_waitcnt":
            c["wait_lgkm"] += "lgkmcnt" in t
            c["wait_vm"] += "vmcnt" in t
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            c["smem"] += 1
        elif op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
            c["branch"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


print(f"{'phase':28s} {'ticks(1 exe)':>12s} {'instr':>6s} {'VALU':>5s} {'SALU':>5s} {'LDS':>4s} {'VMEM':>5s} "
      f"{'SMEM':>5s} {'br':>4s} {'wait lgkm':>9s} {'wait vm':>7s} {'ticks/wait':>10s}")
tot = None
for k0, k1 in zip(order, order[1:]):
    if k0 not in pos or k1 not in pos:
        continue
    c = classify(body[pos[k0]:pos[k1]])
    t = measured.get(SLOT[k0])
    waits = c["wait_lgkm"] + c["wait_vm"]
    tpw = f"{t / waits:10.0f}" if t and waits else f"{'':>10s}"
    print(f"{SLOT[k0] + ' -> ' + SLOT[k1]:28s} {t if t else '':>12} {c['total']:6d} {c['valu']:5d} {c['salu']:5d} "
          f"{c['lds']:4d} {c['vmem']:5d} {c['smem']:5d} {c['branch']:4d} {c['wait_lgkm']:9d} {c['wait_vm']:7d} {tpw}")

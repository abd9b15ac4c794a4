"""Static checks of emitted gfx950 assembly (test infrastructure, CPU only; tests/test_build.py).

The work-queue PageRank kernel (k_pr_pull_units<..., QUEUE=true>) hung twice on the GPU when the
compiler turned the queue fetch's `w >= total` exit into a divergent branch: the other lanes of
wave 0 kept running the loop's barriers (gx_pr_sorted.hip queue_fetch).  These helpers read the
kernel's assembly and find:
- queue_fetch_region(): the fetch (the kernel's first returning global_atomic_add), the two
  barriers that publish its result to the workgroup, and the first conditional branch after
  them, which is the loop exit, with the instruction that set its condition;
- exec_depth(): along the straight-line code from the loop header to that exit, the nesting of
  exec-masked regions (s_and_saveexec_b64 opens one, s_or_b64 exec, exec, sX closes it) at every
  instruction, so a test can require every barrier there to sit at depth 0 (full EXEC)."""
import re


def parse(lines):
    """-> (instructions, label -> index of the next instruction)."""
    ins, labels = [], {}
    for raw in lines:
        t = raw.split(";")[0].rstrip()
        if not t.strip():
            continue
        if not t[0].isspace():
            m = re.match(r"^([\w.$]+):", t)
            if m:
                labels[m.group(1)] = len(ins)
            continue
        t = t.strip()
        if t.startswith("."):
            continue
        ins.append(t)
    return ins, labels


def kernel_body(asm_text, symbol):
    """The lines of one function (its label to .Lfunc_end)."""
    lines = asm_text.splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(symbol + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def queue_fetch_region(ins, labels):
    """-> dict(header, fetch, barriers, cond, exit) as instruction indices (cond may be None),
    or None when the kernel has no returning atomic add."""
    fetch = next((i for i, t in enumerate(ins) if t.startswith("global_atomic_add") and " sc0" in t), None)
    if fetch is None:
        return None
    # the loop header: the last label at or before the fetch that a later branch jumps back to
    back = set()
    for i, t in enumerate(ins):
        m = re.match(r"s_(?:c)?branch\w*\s+(\S+)", t)
        if m and m.group(1) in labels and labels[m.group(1)] <= i:
            back.add(labels[m.group(1)])
    header = max((h for h in back if h <= fetch), default=0)
    bars, cond = [], None
    for i in range(fetch + 1, len(ins)):
        t = ins[i]
        if t.startswith("s_barrier"):
            bars.append(i)
            continue
        if len(bars) < 2:
            continue
        op = t.split()[0]
        if op.startswith("s_cmp") or op.startswith("v_cmp") or op.startswith("s_bitcmp"):
            cond = i
        if op.startswith("s_cbranch"):
            return dict(header=header, fetch=fetch, barriers=bars, cond=cond, exit=i)
    return None


def exec_depth(ins, start, end):
    """Depth of exec-masked regions before each instruction in [start, end), straight-line."""
    d, out = 0, []
    for i in range(start, end):
        out.append(d)
        t = ins[i]
        op = t.split()[0]
        if op.endswith("_saveexec_b64") and not op.startswith("s_or_saveexec"):
            d += 1
        elif re.match(r"s_or_b64 exec, exec, ", t):
            d = max(0, d - 1)
        elif op in ("s_mov_b64", "s_and_b64", "s_andn2_b64", "s_xor_b64") and t.split()[1].rstrip(",") == "exec":
            d += 1   # any other narrowing of EXEC on this path counts as a masked region
    return out

"""Per-basic-block instruction mix of one kernel in a hipcc -S (gfx950)
assembly file: VALU / v_mad_u64_u32 / LDS / VMEM counts and the block's
closing branch, so a kernel's loop body and its divergent side paths can be
priced in issue slots (v_mad_u64_u32 takes two VALU issue slots).

    python tools/isa_blocks.py FILE.s KERNEL_SUBSTRING
"""
import re
import sys


def kernel_lines(path, key):
    out, on = [], False
    for l in open(path):
        if not on and re.match(r"^_Z\S*%s\S*:" % re.escape(key), l):
            on = True
        if on:
            out.append(l.rstrip("\n"))
            if l.startswith(".Lfunc_end"):
                break
    return out


def blocks(lines):
    res, cur = [], None
    for l in lines:
        m = re.match(r"^(\.LBB\S+|_Z\S+):", l)
        if m:
            cur = [m.group(1), []]
            res.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if cur is not None:
            cur[1].append(s.split()[0])
    return res


def main():
    path, key = sys.argv[1], sys.argv[2]
    tot = {"n": 0, "valu": 0, "mad": 0}
    for name, ins in blocks(kernel_lines(path, key)):
        v = sum(1 for i in ins if i.startswith("v_"))
        mad = sum(1 for i in ins if i.startswith("v_mad_u64_u32"))
        ds = sum(1 for i in ins if i.startswith("ds_"))
        vm = sum(1 for i in ins if i.startswith(("global_", "buffer_")))
        br = [i for i in ins if i.startswith("s_cbranch") or i == "s_branch"]
        tot["n"] += len(ins)
        tot["valu"] += v
        tot["mad"] += mad
        print("%-24s n=%5d valu=%5d mad=%4d slots=%5d ds=%3d vmem=%3d %s"
              % (name[:24], len(ins), v, mad, v + mad, ds, vm, br[-1] if br else ""))
    print("total", tot)


if __name__ == "__main__":
    main()

"""Critical-path attribution of the last sqrt-PST open in a rocprofv3 kernel
trace (tools/prof_open.py under --kernel-trace), per MIPP round:

* B (cross terms): the round starts at its k_mipp_weights (after the host
  uploaded the previous challenge); u_l / u_r are ready when B's download
  copy ends;
* A (t_l / t_r): the combination of the look-ahead tables with the
  challenge (k_gt_tab_prod1/2, k_gt_final) and the download of t;
* the look-ahead chains (two alternating queues): fold sets (fbt +
  seg_sum), lines (k_line_pair), line tree (k_chunk_prod), block multipliers,
  Horner + final exponentiation (k_chain_final_rns), squaring tables;
* host: the gap between the later of (u, t) and the next round's upload
  (transcript absorption, challenge, enqueue).
Queues are identified by the kernels they run.

    python tools/open_critical.py run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"tpst::|unsigned int|unsigned long|const|\*|void |Fp<FqCfg>", "", n).split("(")[0].strip()


CLASSES = [("fold", ("k_mipp_scalar_sets", "k_fbt_partial_quad<", "k_seg_sum_quad<")), ("lines", ("k_line_pair",)),
           ("tree", ("k_chunk_prod_rns",)), ("blocks", ("k_miller_blocks_rns",)), ("final_exp", ("k_chain_final_rns",)),
           ("sq_tables", ("k_gt_sq_table_rns",))]


def klass(n):
    for c, keys in CLASSES:
        if any(k in n for k in keys):
            return c
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?"))
                for r in rows)
    # the last open: after the last commit's k_batch_sort
    i0 = max(i for i, e in enumerate(ev) if "k_batch_sort" in e[2])
    j = i0
    while j < len(ev) and "k_chain_final" not in ev[j][2]:
        j += 1
    seg = ev[j + 1:]
    t0 = seg[0][0]
    byq = defaultdict(list)
    for e in seg:
        byq[e[3]].append(e)
    qA = next(q for q, es in byq.items() if any("k_gt_tab_prod1" in e[2] for e in es))
    qB = next(q for q, es in byq.items() if any("k_mipp_weights" in e[2] for e in es) and q != qA)
    qLA = [q for q, es in byq.items() if any("k_gt_sq_table_rns" in e[2] for e in es)]
    ms = lambda x: (x - t0) / 1e6  # noqa: E731
    # rounds: B's k_mipp_weights
    B = byq[qB]
    starts = [e[0] for e in B if "k_mipp_weights" in e[2]]
    A = byq[qA]
    print("open span %.3f ms; queues A=%s B=%s look-ahead=%s" % ((max(e[1] for e in seg) - t0) / 1e6, qA, qB, qLA))
    print("%5s %8s %8s %8s %8s %8s" % ("round", "start", "u_ready", "t_ready", "next", "host"))
    for r, s in enumerate(starts):
        nxt = starts[r + 1] if r + 1 < len(starts) else None
        lim = nxt if nxt else max(e[1] for e in seg)
        ub = [e for e in B if s <= e[0] < lim and "copyBuffer" in e[2]]
        u = ub[0][1] if ub else None
        ta = [e for e in A if s <= e[0] < lim and "copyBuffer" in e[2]]
        t = ta[0][1] if ta else None
        host = (nxt - max(x for x in (u, t) if x)) / 1e6 if nxt and (u or t) else float("nan")
        print("%5d %8.3f %8s %8s %8s %8.3f" % (r, ms(s), "%.3f" % ms(u) if u else "-", "%.3f" % ms(t) if t else "-",
                                               "%.3f" % ms(nxt) if nxt else "-", host))
    print("look-ahead chains (start, end, span; per class: ms)")
    for q in qLA:
        es = byq[q]
        chains, cur = [], []
        for e in es:
            cur.append(e)
            if "k_gt_sq_table_rns" in e[2]:
                chains.append(cur)
                cur = []
        for c in chains:
            tot = defaultdict(float)
            for e in c:
                tot[klass(e[2])] += (e[1] - e[0]) / 1e6
            busy = sum(tot.values())
            span = (c[-1][1] - c[0][0]) / 1e6
            print("q%-3s %8.3f %8.3f %7.3f  %s  gaps %.3f" % (q, ms(c[0][0]), ms(c[-1][1]), span,
                  " ".join("%s %.3f" % (k, tot[k]) for k, _ in CLASSES + [("other", 0)] if tot.get(k)), span - busy))


if __name__ == "__main__":
    main()

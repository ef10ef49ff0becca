"""Per-round gaps of the MIPP open from a rocprofv3 kernel trace: final
exponentiation (k_chain_final, two groups) end -> next one's start, and end ->
the next host-to-device copy on the same queue (= host transcript time).
    python tools/open_gaps.py gpurun_out/<tag>/prof/run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ch = [r for r in rows if "k_chain_final" in r["Kernel_Name"] and r["Grid_Size_X"] == "128"]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ch, ch[1:])]
gaps = [g for g in gaps if g < 2000]
host = []
for a in ch[:60]:
    te = int(a["End_Timestamp"])
    nxt = [r for r in rows if r["Queue_Id"] == a["Queue_Id"] and int(r["Start_Timestamp"]) > te + 20000
           and "copyBuffer" in r["Kernel_Name"]][:1]
    if nxt and (int(nxt[0]["Start_Timestamp"]) - te) / 1e3 < 1500:
        host.append((int(nxt[0]["Start_Timestamp"]) - te) / 1e3)
print("final-exp -> final-exp gap median %.0f us over %d rounds; host transcript gap median %.0f us over %d"
      % (statistics.median(gaps), len(gaps), statistics.median(host), len(host)))

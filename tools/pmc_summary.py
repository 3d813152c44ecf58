"""Aggregate rocprofv3 --pmc CSVs (gpurun_out/pmc*/run_counter_collection.csv)
for one kernel:  python tools/pmc_summary.py 'lean_tile<false, false, true>' [cells]"""
import collections
import csv
import glob
import sys


def main():
    pat = sys.argv[1]
    cells = float(sys.argv[2]) if len(sys.argv) > 2 else 400000.0
    out = {}
    for f in sorted(glob.glob(sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/pmc*/run_counter_collection.csv")):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            out[k] = sum(v) / len(v)
    print("| counter | per dispatch | per cell |\n|---|---:|---:|")
    for k in sorted(out):
        print("| %s | %.4g | %.4g |" % (k, out[k], out[k] / cells))
    if "SQ_INSTS_VALU" in out:
        print("\nVALU instr / cell: %.0f" % (out["SQ_INSTS_VALU"] * 64 / cells))
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        rd, wr = out["FETCH_SIZE"] * 2048, out["WRITE_SIZE"] * 1024
        print("HBM read ~%.1f MB (2 x FETCH_SIZE), write %.1f MB, %.0f B/cell" % (rd / 1e6, wr / 1e6, (rd + wr) / cells))
    if "SQ_WAVE_CYCLES" in out:
        w = out["SQ_WAVE_CYCLES"]
        print("wave cycles: wait %.0f%%  issue-stall %.0f%%  active %.0f%%" % (
            100 * out.get("SQ_WAIT_ANY", 0) / w, 100 * out.get("SQ_WAIT_INST_ANY", 0) / w,
            100 * out.get("SQ_ACTIVE_INST_ANY", 0) / w))
    if "GRBM_GUI_ACTIVE" in out:
        print("GRBM_GUI_ACTIVE/8 = %.0f cycles" % (out["GRBM_GUI_ACTIVE"] / 8))


if __name__ == "__main__":
    main()

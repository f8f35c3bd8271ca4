"""Fold gpurun_out/pmc_<cfg>.json (scripts/pmc_summarize.py) into
profiles/pmc_summary.json, the per-config HBM traffic bench.py reports as
roofline.traffic, and copy each file to profiles/<tag>_pmc_<cfg>.json.
usage: python scripts/pmc_to_summary.py TAG CFG [CFG ...]   (host)"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, cfgs = sys.argv[1], sys.argv[2:]
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    with open(path) as fh:
        summ = json.load(fh)
    for cfg in cfgs:
        src = os.path.join(ROOT, "gpurun_out", f"pmc_{cfg}.json")
        dst = os.path.join(ROOT, "profiles", f"{tag}_pmc_{cfg}.json")
        shutil.copyfile(src, dst)
        with open(src) as fh:
            r = json.load(fh)
        P, A, O = cfg.split("x")
        summ[f"P{P}_A{A}_O{O}"] = {
            "hbm_bytes_per_launch": r["hbm_bytes_per_launch_corrected"],
            "fetch_size_kib": r["FETCH_SIZE"],
            "write_size_kib": r["WRITE_SIZE"],
            "wait_any_over_wave_cycles": r["SQ_WAIT_ANY"] / r["SQ_WAVE_CYCLES"],
            "valu_per_wave": r["SQ_INSTS_VALU"] / r["SQ_WAVES"],
            "correction": "(2*FETCH_SIZE + WRITE_SIZE)*1024: gfx950 FETCH_SIZE reports half of a "
                          "wide coalesced read (MI355X_MICROARCH.md HBM section); WRITE_SIZE exact "
                          "for 16-B/lane stores",
            "source": f"profiles/{tag}_pmc_{cfg}.json (scripts/pmc_collect.sh: separate --pmc "
                      f"passes with --kernel-trace only; committed measurement, not taken in the "
                      f"bench run)",
        }
    with open(path, "w") as fh:
        json.dump(summ, fh, indent=1, sort_keys=True)
        fh.write("\n")
    print("updated", path, "with", cfgs)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""MFMA-busy fraction per kernel from a folded --pmc pass (scripts/pmc_summary.py output).

Usage: mfma_busy.py CONFIG PMC.json

  cycles     = GRBM_GUI_ACTIVE / 8          (rocprofv3 sums the GPU clock over the 8 XCDs;
                                              MI355X_MICROARCH.md, DVFS give-back)
  busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
  cyc/inst   = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA: the SIMD-cycles one MFMA keeps the
               matrix core busy (32 for v_mfma_f32_16x16x4_f32 at 64 f32 FLOP/SIMD/cycle);
               it checks that the busy counter is summed over SIMDs as busy_frac assumes.
GRBM_GUI_ACTIVE includes the dispatch ramp of the launch, so on launches of ~10 us
busy_frac is the fraction of the WHOLE launch the matrix cores were busy.
"""
import json
import sys

N_SIMD = 1024


def main():
    cfg, path = sys.argv[1], sys.argv[2]
    d = json.load(open(path))
    print(f"== {cfg}: MFMA-busy per launch (averaged over launches)")
    print(f"{'kernel':70s} {'launches':>8s} {'cycles':>9s} {'mfma_insts':>11s} {'busy_cyc':>12s} {'cyc/inst':>8s} {'busy_frac':>9s}")
    tot_busy = tot_cyc = 0.0
    for k, v in sorted(d.items()):
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in v or "GRBM_GUI_ACTIVE" not in v:
            continue
        busy, insts = v["SQ_VALU_MFMA_BUSY_CYCLES"], v.get("SQ_INSTS_MFMA", 0.0)
        cyc = v["GRBM_GUI_ACTIVE"] / 8.0
        if insts <= 0:
            continue
        frac = busy / (N_SIMD * cyc) if cyc > 0 else 0.0
        tot_busy += busy
        tot_cyc += cyc
        print(f"{k[:70]:70s} {v['launches']:8d} {cyc:9.0f} {insts:11.0f} {busy:12.0f} {busy / insts:8.1f} {frac:9.4f}")
    if tot_cyc > 0:
        print(f"{'all MFMA kernels (one launch each)':70s} {'':8s} {tot_cyc:9.0f} {'':11s} {tot_busy:12.0f} {'':8s} {tot_busy / (N_SIMD * tot_cyc):9.4f}")


if __name__ == "__main__":
    main()

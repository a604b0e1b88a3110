"""Per-phase SQ counters of k_encode_rows by differencing phase-repeat builds.

  python tools/enc_phase_sq.py --build            # the variant libraries (CPU)
  python tools/enc_phase_sq.py gpurun_out/encphase [out.json]

A build with -DWG_EXP_REP_<PHASE>=2 runs that phase twice per macroblock;
the phase is idempotent, so the outputs are unchanged and (build - default)
is one execution of the phase with the launch's real data flow.  Per phase
and macroblock: wave-cycles, VALU instructions, mean active lanes per VALU
instruction (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU), LDS bank-conflict
cycles and their share of the phase's LDS-active cycles, and the wave's
waiting cycles (SQ_WAIT_ANY, parked on s_waitcnt / s_sleep) and issue
stalls (SQ_WAIT_INST_ANY).  SQ_WAVE_CYCLES, SQ_ACTIVE_INST_VALU, SQ_WAIT_*
count 4-cycle units on gfx950 (x4 below, as profiles/r04_enc_sq.json used)."""
import json
import os
import subprocess
import sys

PHASES = {"RD": "I16 + UV RD", "I4": "I4 RD (all steps)", "PRE": "I4 value table + pre-screen",
          "CAND": "I4 candidates: prediction + FTransform", "PREP": "I4 trellis position records",
          "DP": "I4 trellis DP", "FIN": "final residuals (I16 trellis rounds, chroma)"}
N_MB = 64 * 120 * 68  # one 64 x 1080p launch


def build():
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webp_amd")
    for p in PHASES:
        subprocess.run(["make", "-s", "-j8", "-C", root, "variant", "NAME=rep" + p, "DEFS=-DWG_EXP_REP_%s=2" % p],
                       check=True)


def per_mb(rec):
    r = rec["k_encode_rows"]
    return {
        "wave_cycles": 4 * r["SQ_WAVE_CYCLES"] / N_MB,
        "valu_insts": r["SQ_INSTS_VALU"] / N_MB,
        "valu_cycles": 4 * r["SQ_ACTIVE_INST_VALU"] / N_MB,
        "valu_thread_cycles": r["SQ_THREAD_CYCLES_VALU"] / N_MB,
        "lds_bank_conflict": r["SQ_LDS_BANK_CONFLICT"] / N_MB,
        "lds_active": r["SQ_LDS_IDX_ACTIVE"] / N_MB,
        "wait_any": 4 * r["SQ_WAIT_ANY"] / N_MB,
        "wait_inst_any": 4 * r["SQ_WAIT_INST_ANY"] / N_MB,
    }


def derived(d):
    out = {k: round(v, 1) for k, v in d.items()}
    out["active_lanes_per_valu"] = round(d["valu_thread_cycles"] / d["valu_cycles"] * 4, 2) if d["valu_cycles"] else None
    out["bank_conflict_share"] = round(d["lds_bank_conflict"] / d["lds_active"], 3) if d["lds_active"] else None
    return out


def out_hash():
    """sha256 of the wg_mb_enc records + reconstruction of three mixed 1080p
    frames with the library WEBPGPU_LIB names (the repeat builds must equal
    the default)."""
    import hashlib

    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools import synth
    from webp_amd import frames
    w, h = 1920, 1080
    rgba = np.stack([synth.gradient_rgba(w, h), synth.noise_rgba(w, h, seed=3), synth.blobs_rgba(w, h, seed=3)])
    out, (ry, ru, rv), _, _, _ = frames.encode_frames(torch.from_numpy(rgba).cuda())
    torch.cuda.synchronize()
    hs = hashlib.sha256()
    for t in (out, ry, ru, rv):
        hs.update(t.cpu().numpy().tobytes())
    print(os.environ.get("WEBPGPU_LIB", "default"), hs.hexdigest())


def main(argv):
    if argv and argv[0] == "--build":
        return build()
    if argv and argv[0] == "--hash":
        return out_hash()
    d = argv[0]
    base = per_mb(json.load(open(os.path.join(d, "sq_base.json"))))
    res = {"units": "per macroblock of one 64 x 1080p k_encode_rows launch (mixed gradient / noise / blobs, q75 "
                    "defaults); phase = (phase-repeat build - default build)",
           "whole_kernel": derived(base), "phases": {}}
    for p, name in PHASES.items():
        f = os.path.join(d, "sq_%s.json" % p)
        if not os.path.exists(f):
            continue
        v = per_mb(json.load(open(f)))
        res["phases"][p] = dict(name=name, **derived({k: v[k] - base[k] for k in base}))
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(argv) > 1:
        open(argv[1], "w").write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])

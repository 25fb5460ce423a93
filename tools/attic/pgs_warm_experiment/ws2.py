"""Convergence of warm-started PGS inside a control step vs cold 8 sweeps, per robot (drive.run)."""
import sys
from drive import run, lib
import ctypes as C
lib.exp_omega.argtypes = [C.c_float]; lib.exp_omega(1.0)
task = sys.argv[1]; N = int(sys.argv[2]); steps = int(sys.argv[3])
for cold, wsw, warm, persist in [(8, 8, 0, 0), (8, 6, 1, 0), (8, 5, 1, 0), (8, 4, 1, 0)]:
    r = run(task, N, steps, cold, wsw, warm, persist, ref=200)
    print(f"{task} cold={cold} warm_sw={wsw} warm={warm} persist={persist}: sweeps {r['sweeps']:.2f} v_rms {r['v_rms']:.2e} v_max {r['v_max']:.2e} lam_rel {r['lam_err']/max(r['lam_mag'],1e-12):.3e} energy {r['energy']:.2e} P>1cm {r['frac_vmax_gt_1cm']:.3f} falls {r['falls']}", flush=True)

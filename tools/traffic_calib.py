"""Known-byte calibration of the rocprofv3 traffic counters for the fused env step's own
access pattern (MI355X_MICROARCH.md §HBM: "Other access widths are uncalibrated: calibrate
on a known byte count in your own access pattern before trusting an absolute").

The I/O-only diagnostic build (make -C unitree-rl-gym_amd/csrc iodiag: LGS_DIAG_IO_ONLY, the
physics substep removed) issues exactly the step's global loads and stores -- the per-env
rows listed below, read and written once per control step, plus a few uniform words -- so
its FETCH_SIZE / WRITE_SIZE per launch against these known bytes is the counters' tally
factor for this pattern.  The shipped kernel's counters divided by those factors are its
HBM bytes.  (The 1 GiB float4 copy calibration of tools/pmc_summary.py -- FETCH_SIZE = half
the bytes of a wide streaming read -- does not carry over: the step's rows are 4-96 B
pieces of 128-B lines.)

usage: python tools/traffic_calib.py <pmc_k_step.json> <pmc_k_step_io_only.json> <num_envs> <out.json>
(Go2: A = D = 12, B = 19 bodies, F = 4 feet, O = 48 observations, 10 reward terms, no priv)
"""
import json
import sys


def go2_io_bytes(A=12, D=12, B=19, F=4, O=48, nR=10):
    """Per env and control step: every global row k_step reads and writes (Go2 layout)."""
    f = 4
    read = {"actions_in": A * f, "last_dof_vel": D * f, "root_states": 13 * f, "dof_state": 2 * D * f,
            "friction + added_mass": 2 * f, "commands": 4 * f, "episode_length": 8, "last_actions": A * f,
            "feet_air_time": F * f, "last_contacts": F, "episode_sums": nR * f}
    write = {"actions (clipped copy)": A * f, "root_states": 13 * f, "dof_state": 2 * D * f,
             "net_contact_forces": 3 * B * f, "torques": D * f, "commands[2] (heading)": f, "episode_length": 8,
             "base_lin_vel + base_ang_vel + projected_gravity + rpy": 12 * f, "phase + leg_phase": 3 * f,
             "rew": f, "reset + time_out": 2, "episode_sums": nR * f, "feet_air_time": F * f, "last_contacts": F,
             "obs": O * f, "last_actions": A * f, "last_dof_vel": D * f, "last_root_vel": 6 * f,
             "push bookkeeping (vsim)": 2 * f}
    return read, write


def main(full_json, io_json, n, out):
    n = int(n)
    full, io = json.load(open(full_json)), json.load(open(io_json))
    rd, wr = go2_io_bytes()
    kr, kw = sum(rd.values()) * n, sum(wr.values()) * n
    fr_io, fw_io = io["fetch_size_kib"] * 1024.0, io["write_size_kib"] * 1024.0
    fr, fw = full["fetch_size_kib"] * 1024.0, full["write_size_kib"] * 1024.0
    sr, sw = kr / fr_io, kw / fw_io  # bytes per counted byte, for this access pattern
    res = {
        "num_envs": n,
        "known_bytes_per_env": {"read": rd, "write": wr, "read_total": sum(rd.values()),
                                "write_total": sum(wr.values())},
        "io_only_build": {"fetch_size_bytes": fr_io, "write_size_bytes": fw_io, "known_read_bytes": kr,
                          "known_write_bytes": kw, "read_scale": sr, "write_scale": sw,
                          "avg_ns": io.get("avg_ns")},
        "k_step": {"fetch_size_bytes": fr, "write_size_bytes": fw, "avg_ns": full.get("avg_ns"),
                   "read_bytes_per_launch": fr * sr, "write_bytes_per_launch": fw * sw,
                   "hbm_bytes_per_launch": fr * sr + fw * sw,
                   "copy_calibrated_bytes_per_launch": full.get("hbm_bytes_per_launch")},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["io_only_build"]), json.dumps(res["k_step"]))


if __name__ == "__main__":
    main(*sys.argv[1:5])

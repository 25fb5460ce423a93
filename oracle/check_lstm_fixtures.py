"""Pins the recurrent-policy fixtures (tests/golden/lstm_policy_<robot>.npz) to the reference's
archives, deploy/pre_train/<robot>/motion.pt, without loading them: a TorchScript archive is a
zip whose tensors are raw little-endian storages (`<archive>/data/<i>`), numbered in the order
the module's state was serialized.  Nothing from the archive is unpickled or executed: the zip
directory is listed and those raw byte entries are read.

For each robot the fixture keeps the module's state order (hidden_state, cell_state,
actor.0.weight, actor.0.bias, actor.2.weight, actor.2.bias, memory.weight_ih_l0,
memory.weight_hh_l0, memory.bias_ih_l0, memory.bias_hh_l0), and the archive holds exactly those
storages:
  * every parameter equals, byte for byte, the storage at its position;
  * the two memory buffers are zeros in the archive (the exporter's reset state) and, in the
    fixture, the state the extraction left behind: that of the 5-step run after reset_memory(),
    which nn.LSTM reproduces from the fixture's own weights and inputs (1e-5).
The fixture's outputs are then re-derived from those weights with torch's nn.LSTM by
tests/test_rsl_rl.py (CPU) and through the HIP LSTM by tests/test_gpu_recurrent.py.

Test infrastructure (tests/test_golden_lstm_archive.py); reads /root/reference, so it runs in
the build container only.

usage: python oracle/check_lstm_fixtures.py [reference_root]"""
import os
import sys
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")
ROBOTS = ("g1", "h1", "h1_2")


def storages(archive):
    """{index: raw bytes} of the archive's tensor storages (zip entries '<top>/data/<i>')."""
    out = {}
    with zipfile.ZipFile(archive) as z:
        for name in z.namelist():
            head, _, leaf = name.rpartition("/")
            if head.endswith("/data") and leaf.isdigit():
                out[int(leaf)] = z.read(name)
    return out


def check(reference_root, robot):
    """Returns a list of mismatch descriptions (empty: the fixture is the archive's weights)."""
    fx = np.load(os.path.join(GOLDEN, f"lstm_policy_{robot}.npz"))  # arrays only (allow_pickle=False)
    weights = [k for k in fx.files if k.startswith("w.")]
    st = storages(os.path.join(reference_root, "deploy", "pre_train", robot, "motion.pt"))
    bad = []
    if sorted(st) != list(range(len(weights))):
        bad.append(f"{robot}: archive storages {sorted(st)} vs {len(weights)} fixture weights")
    state = ("w.hidden_state", "w.cell_state")
    for i, k in enumerate(weights):
        a = np.ascontiguousarray(fx[k], dtype="<f4").tobytes()
        if k in state:
            if st.get(i) != bytes(len(a)):
                bad.append(f"{robot}: archive storage {i} ({k}) is not the zero reset state")
        elif st.get(i) != a:
            bad.append(f"{robot}: {k} != archive storage {i} ({len(a)} vs {len(st.get(i, b''))} bytes)")
    import torch  # the memory's state after the fixture's 5-step post-reset run
    lstm = torch.nn.LSTM(fx["w.memory.weight_ih_l0"].shape[1], fx["w.memory.weight_hh_l0"].shape[1], 1)
    lstm.load_state_dict({k[len("w.memory."):]: torch.from_numpy(fx[k]) for k in weights if k.startswith("w.memory.")})
    with torch.no_grad():
        _, (h, c) = lstm(torch.from_numpy(fx["inputs"][:5])[:, None, :])
    for k, v in zip(state, (h, c)):
        if not np.allclose(v.numpy(), fx[k], rtol=1e-5, atol=1e-5):
            bad.append(f"{robot}: {k} is not the state after the 5-step post-reset run")
    return bad


def main(reference_root):
    bad = [m for r in ROBOTS for m in check(reference_root, r)]
    for m in bad:
        print(m)
    if not bad:
        print(f"{', '.join(ROBOTS)}: every fixture parameter equals its archive storage byte for byte; "
              "the memory states are the 5-step post-reset run's")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference"))

"""A bounded in-kernel wait that gives up must be loud.

The split-role DeepFM kernel (deepfm_ws) hands the gathered row bursts from
its loader waves to its compute waves through LDS counters, each wait bounded.
The diagnostic build (scripts/build_diag.sh, -DRS_DIAG_STAMPS) has a knob,
RS_ABLATE bit 32, under which the loaders never signal the second burst: the
compute waves' wait must time out, set RS_FLAG_TIMEOUT, let the grid drain,
and the checked forward must raise RSError (never return the stale output).
Runs in a child process (the diagnostic library, an env knob); skipped when
the diagnostic library is not in the tree (it is built and shipped for stamp
sessions only) or older than any kernel source or header (a stale build would
pass against kernels that predate the tree)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
DIAG = ROOT / "recommender_system_amd" / "librs_hip_diag.so"

CHILD = r'''
import sys
from pathlib import Path
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
from recommender_system_amd import _lib
_lib._LIB_PATH = Path(sys.argv[2])
_lib._ALLOW_MISSING = True  # the diagnostic build may predate entries this test does not call
import recommender_system_amd as rs
from tests.helpers import criteo_columns, random_ids
rng = np.random.default_rng(0)
vocabs = rng.integers(2, 3000, size=26)
m = rs.DeepFM(criteo_columns(vocabs, embed_dim=16), 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=16, seed=1)
_lib.set_option(_lib.OPT_DEEPFM_KERNEL, 0)
ids = torch.as_tensor(random_ids(rng, 64, vocabs, np.int32), device="cuda")
dense = torch.rand(64, 13, device="cuda")
try:
    m.forward_fused((dense, ids))
    print("NO-RAISE")
except _lib.RSError as e:
    print("RSERROR", e)
'''


@pytest.mark.gpu
def test_deepfm_ws_wait_timeout_raises(gpu):
    if not DIAG.exists():
        pytest.skip("diagnostic library not built/shipped (scripts/build_diag.sh)")
    srcs = [f for d in (ROOT / "recommender_system_amd" / "csrc", ROOT / "include") for f in d.iterdir()
            if f.suffix in (".hip", ".hpp", ".cpp", ".h")]
    newest = max(srcs, key=lambda f: f.stat().st_mtime)
    if newest.stat().st_mtime > DIAG.stat().st_mtime:
        pytest.skip(f"diagnostic library older than {newest.name}: rebuild it (scripts/build_diag.sh, or "
                    f"RS_BUILD_DIAG=1 with __graft_entry__.build()) - a stale build would test old kernels")
    env = dict(os.environ, RS_ABLATE="32")
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(DIAG)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "RSERROR" in r.stdout and "RS_FLAG_TIMEOUT" in r.stdout, r.stdout + r.stderr[-2000:]

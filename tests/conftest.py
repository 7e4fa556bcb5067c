"""pytest configuration: registers the `gpu` marker and puts the package dir on sys.path.

`-m "not gpu"` runs on CPU only (oracle vs golden fixtures, host logic, C-ABI symbol export);
`-m gpu` runs the HIP parity tests on an MI355X.
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vision-pt_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libvpt_hip.so")

import os
import sys

# GPU_MAX_HW_QUEUES is left as the environment has it (HIP's default 4 on the
# GPU boxes): the suite runs the library's default deployment; the tests that
# need a specific value set it in a fresh process (test_gpu_parity.py,
# test_gpu_realrccl.py: ..._live_at_hip_default_hw_queues).

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); run with -m gpu on the GPU box")

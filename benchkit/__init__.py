"""Measurement helpers of bench.py (the headline line's extras): host CPU
facts, host-inclusive (PCIe) legs, device-resident side legs, and the
rocprofv3 child passes. Test and measurement infrastructure only -- nothing
here is on the product path, and nothing here imports oracle/ (bench.py's
own cpu_baseline leg is the only bench code that does)."""
import os

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED_BASE = 0x5709B
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")

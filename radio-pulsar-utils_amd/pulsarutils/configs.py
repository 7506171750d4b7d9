"""Benchmark / parity configurations C1-C5 (BASELINE.json ``configs``).

Each config names a filterbank shape, its band and sampling time, and a DM range
chosen so that the reference's own ``dedispersion_plan``
(``pulsarutils/dedispersion.py:149-171``) yields exactly the stated trial count.
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Config:
    name: str
    nchan: int
    nsamples: int
    dtype: str          # "f64" | "f32" | "u8"
    start_freq: float   # MHz, lower edge of channel 0 (reference convention)
    bandwidth: float    # MHz
    tsamp: float        # s
    dmmin: float
    dmmax: float
    ntrials: int        # expected len(dedispersion_plan(...))
    pulse_dm: float
    seed: int


CONFIGS = {
    # simulate.py pulsar, numpy reference on CPU
    "C1": Config("C1", 64, 1 << 16, "f64", 1200.0, 200.0, 5e-4,
                 100.0, 164.4285, 100, 130.0, 2024),
    # the single-GPU headline config (BASELINE.json configs[1])
    "C2": Config("C2", 1024, 1 << 20, "f32", 1200.0, 300.0, 64e-6,
                 0.0, 61.609062, 1000, 40.0, 2025),
    # 8-bit, sharded over 8 GPUs (configs[2])
    "C3": Config("C3", 4096, 1 << 22, "u8", 1200.0, 300.0, 64e-6,
                 0.0, 308.415522, 5000, 200.0, 2026),
    # RFI-heavy cleaning config (configs[3]); 100 trials for the search leg
    "C4": Config("C4", 1024, 1 << 18, "f32", 1200.0, 300.0, 64e-6,
                 30.0, 36.077609, 100, 33.0, 2027),
    # LOFAR-like low band: shift spread > time tile (configs[4])
    "C5": Config("C5", 256, 1 << 17, "f32", 110.0, 80.0, 1e-3,
                 10.0, 12.18677, 500, 11.0, 2028),
}

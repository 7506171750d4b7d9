"""pulsarutils (MI355X-native): drop-in dedispersion + RFI-cleaning hot path.

Same public API as the reference ``pulsarutils.dedispersion`` / ``pulsarutils.clean`` /
``pulsarutils.stats`` (matteobachetti/radio-pulsar-utils), computed by hand-written
HIP kernels for gfx950 (``csrc/``) behind a C-ABI (``include/pulsarutils_hip.h``).
"""
__version__ = "0.1.0"

"""liteasr_amd: MI355X-native U2 / Conformer + hybrid CTC-attention training path.

Drop-in for the hot path of Nazukixv/LiteASR: same registries (task=/model=/criterion=/
optimizer=), same config schema, same state_dict, same call conventions; the compute is
hand-written HIP for gfx950 (libliteasr_hip.so, C ABI in include/liteasr_hip.h).
"""

__version__ = "0.1.0"

"""daclip_amd — MI355X-native DA-CLIP + IR-SDE inference hot path.

Host-side mirror of the reference's Python API (open_clip.create_model_from_pretrained,
DaCLIP.encode_image(control=True), IRSDE, create_model/DenoisingModel) on top of the
C-ABI library libdaclip_hip.so (csrc/, include/daclip_hip.h).
"""
__version__ = "0.1.0"

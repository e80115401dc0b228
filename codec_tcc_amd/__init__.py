"""codec_tcc_amd -- MI355X-native (gfx950) implementation of wesleyfn/codec-tcc's
LSB bit-plane embed/extract pixel path.  See DESIGN.md and INTEGRATION.md.

Batched API (torch tensors in HBM):   Codec, encode, decode, decode_ref_compat
Reference drop-ins (numpy in/out):    codec_tcc_amd.api (same names as src/codec.py)
"""
from .codec import Codec, Encoded, Payloads, decode, decode_ref_compat, encode, make_payloads, meta_dict, meta_records
from .framing import distribute_message_segments, message_to_bits

__all__ = [
    "Codec", "Encoded", "Payloads", "encode", "decode", "decode_ref_compat", "make_payloads",
    "meta_records", "meta_dict", "message_to_bits", "distribute_message_segments",
]

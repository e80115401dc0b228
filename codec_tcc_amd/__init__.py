"""codec_tcc_amd -- MI355X-native (gfx950) implementation of wesleyfn/codec-tcc's
embed/extract pixel path: the reference's LSB bit-plane scheme (bit-exact with
src/codec.py) and the MED-PEE scheme the north star names.  See DESIGN.md and
INTEGRATION.md.

Batched API (torch tensors in HBM):   encode(covers, payloads, method="lsb"|"pee", ...),
                                      decode(enc), decode_ref_compat, Codec, PeeCodec
Reference drop-ins (numpy in/out):    codec_tcc_amd.api (same names as src/codec.py)
"""
from .codec import Codec, Encoded, Payloads, decode, decode_ref_compat, encode, make_payloads, meta_dict, meta_records
from .framing import distribute_message_segments, message_to_bits
from .pee import PeeCodec, PeeEncoded

__all__ = [
    "Codec", "Encoded", "Payloads", "encode", "decode", "decode_ref_compat", "make_payloads",
    "meta_records", "meta_dict", "message_to_bits", "distribute_message_segments", "PeeCodec", "PeeEncoded",
]

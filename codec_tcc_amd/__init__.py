"""codec_tcc_amd: MI355X-native LSB bit-plane embed/extract."""

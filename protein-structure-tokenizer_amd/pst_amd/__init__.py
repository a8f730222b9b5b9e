"""pst_amd — MI355X-native structure tokenizer (encoder → FSQ token ids).

Host-side mirror of the reference's tokenize path (`scripts/inference_runner.py`,
`structure_tokenizer/data/*`) driving the HIP library `libpst.so` through its C ABI
(`include/pst.h`).
"""
__version__ = "0.1.0"

"""iggy_amd — MI355X-native message-batch codec for Apache Iggy.

The product is the HIP library iggy_amd/libiggy_codec.so behind the C ABI in
include/iggy_codec.h; iggy_amd.codec is its Python host binding.
"""

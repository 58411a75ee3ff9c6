"""iggy_amd — MI355X-native message-batch codec for Apache Iggy.

The product is the HIP library iggy_amd/libiggy_codec.so behind the C ABI in
include/iggy_codec.h; iggy_amd.codec is its Python host binding.

No HIP runtime setting is required. The codec never hands pageable caller memory to
the runtime's copy engine (it stages such bytes through its own pinned chunks, see
host_mem.hpp put_host / get_host and DESIGN.md §8), so its host entry points are
correct with the runtime's defaults, whatever initialised the runtime first.
"""

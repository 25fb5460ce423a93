"""leggedsim: MI355X-native articulated legged-robot simulator (HIP) + model builder.

The C ABI is include/leggedsim.h; `native` loads libleggedsim.so, `model`
builds articulations from URDF, `cabi` mirrors the ABI structs.
"""

"""dformer_amd — MI355X-native (gfx950) DFormer RGB-D encoder Block + ham/MLP decoders.

The compute path is libdformer_hip.so (hand-written HIP kernels behind the C ABI in
include/dformer_hip.h); the nn.Modules keep the reference's constructor arguments, forward()
surfaces and state_dict keys (Originofamonia/DFormer models/encoders/DFormer.py,
models/decoders/ham_head.py, models/decoders/MLPDecoder.py, models/builder.py).
"""
__version__ = "0.1.0"

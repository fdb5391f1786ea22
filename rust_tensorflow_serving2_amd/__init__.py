"""rust_tensorflow_serving2_amd — an MI355X-native TensorFlow-Serving-compatible
model server and client.

Speaks the ``tensorflow.serving`` gRPC API the reference Rust/tonic client
(simonrw/rust-tensorflow-serving2) wraps; executes SavedModels with
hand-written CDNA4 (gfx950) HIP kernels; scales one process per GPU.

Packages: ``client`` (reference API), ``server`` (services, manager, batching,
transports), ``savedmodel`` (SavedModel / TensorBundle I/O), ``graph`` (IR,
reference ops, fusion passes), ``ops`` (HIP kernel bindings), ``models``
(synthetic exporters), ``parallel`` (multi-GPU replicas over RCCL), ``utils``.
"""
__version__ = "0.1.0"

"""MI355X-native MIND embed -> pool -> score hot path.

Host side mirrors the reference package ``news_rec_utils`` module by module
(config, data_utils, modeling_utils, latent_attention, data_model_helper,
evaluation, pipeline, components); the compute runs in hand-written gfx950
HIP kernels in ``libnewsrec_hip.so`` (C-ABI: include/newsrec.h), bound by
``_lib`` and wrapped by ``ops``.  ``import news_rec_utils`` resolves to this
package (see news_rec_utils/__init__.py).
"""
__version__ = "0.1.0"

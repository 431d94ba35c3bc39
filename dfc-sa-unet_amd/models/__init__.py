"""Model package (drop-in for the reference's models/; see models/model_factory.py).

Unlike the reference (whose models/__init__.py imports a module that does not exist), this
package imports cleanly.
"""
from models.unet_dfc_sa_res import LightSelfAttention, DynamicFusionConvAttnBlock, UNetDFCSA, UNetDFCSARes
from models.unet import UNet
from models.unet_dfc_sa_ablation_attention import FullResAttnDFCBlock, FullResolutionAttention, UNet_FullResAttention
from models.model_factory import ModelFactory

__all__ = ["LightSelfAttention", "DynamicFusionConvAttnBlock", "UNetDFCSA", "UNetDFCSARes", "UNet",
           "FullResolutionAttention", "FullResAttnDFCBlock", "UNet_FullResAttention", "ModelFactory"]

"""ModelFactory: config dict -> model (drop-in for the reference's models/model_factory.py:14-186).

Same two entry points (``ModelFactory.get_model(config)`` and
``ModelFactory(config).create_model()``), same defaults (in 3, out 1, features
[64,128,256,512], pool_size 8, ablation_on_qk_channels 8) and the same errors (ValueError
when no config is given or the model name is unknown).  Optional new keys (ignored by the
reference, so unchanged yamls still run): ``model.precision`` / ``training.precision``
('bf16' default, 'fp32').

Built on the MI355X path: 'DFC-SA-Res-Block' (UNetDFCSARes, the north-star model), 'UNet'
(config 1, model_factory.py:94-100), 'UNet_FullResAttention' (config 5, :174-175),
'TransformerUNet'/'TransUNet' (config 4, :113-137) and the ablation zoo (:162-187: UNet_Baseline,
UNet_AttentionOnly, UNet_AdditionFusion, UNet_ConcatFusion, UNet_EncoderOnlyDFC,
UNet_DecoderOnlyDFC, UNet_BothStandardConv, with the reference's argument lists).  The plain ViT
('VisionTransformerSegmentation') raises NotImplementedError.

Pretrained weights are loaded with torch.load(weights_only=True) (a state_dict needs nothing
else); as in the reference a failure is reported and not raised.
"""
import torch

from models.transformer_unet import TransUNet, get_r50_b16_config
from models.unet import UNet
from models.unet_dfc_sa_ablation_attention import UNet_FullResAttention
from models.unet_dfc_sa_ablation_branches import UNet_AttentionOnly, UNet_Baseline
from models.unet_dfc_sa_ablation_fusion import UNet_AdditionFusion, UNet_ConcatFusion
from models.unet_dfc_sa_ablation_placement import UNet_BothStandardConv, UNet_DecoderOnlyDFC, UNet_EncoderOnlyDFC
from models.unet_dfc_sa_res import UNetDFCSARes

# reference :160-187 -- (class, takes pool_size)
_ZOO = {"UNet_Baseline": (UNet_Baseline, False), "UNet_AttentionOnly": (UNet_AttentionOnly, True),
        "UNet_AdditionFusion": (UNet_AdditionFusion, True), "UNet_ConcatFusion": (UNet_ConcatFusion, True),
        "UNet_EncoderOnlyDFC": (UNet_EncoderOnlyDFC, True), "UNet_DecoderOnlyDFC": (UNet_DecoderOnlyDFC, True),
        "UNet_BothStandardConv": (UNet_BothStandardConv, False)}
_BUILT = ("DFC-SA-Res-Block", "UNet", "UNet_FullResAttention", "TransformerUNet", "TransUNet", *_ZOO)
_REFERENCE_ONLY = {"VisionTransformerSegmentation"}


class ModelFactory:
    def __init__(self, config=None):
        self.config = config

    def create_model(self, config=None):
        if config is None:
            if self.config is None:
                raise ValueError("必須提供配置")
            config = self.config
        return ModelFactory._create_model_impl(config)

    @staticmethod
    def get_model(config):
        model = ModelFactory._create_model_impl(config)
        path = config["model"].get("pretrained_path")
        if path:
            try:
                model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
                print(f"成功載入預訓練權重: {path}")
            except Exception as e:  # the reference prints and continues (model_factory.py:69-70)
                print(f"載入預訓練權重失敗: {e}")
        return model

    @staticmethod
    def _create_model_impl(config):
        m = config["model"]
        name = m["name"]
        in_channels = m.get("in_channels", 3)
        out_channels = m.get("out_channels", 1)
        features = m.get("features", [64, 128, 256, 512])
        pool_size = m.get("pool_size", 8)
        qk = m.get("ablation_on_qk_channels", 8)
        precision = m.get("precision", config.get("training", {}).get("precision"))
        if name == "UNet":  # features / pool_size are ignored, as in the reference (:94-100)
            return UNet(n_channels=in_channels, n_classes=out_channels, bilinear=m.get("bilinear", False),
                        precision=precision)
        if name == "DFC-SA-Res-Block":
            return UNetDFCSARes(in_channels=in_channels, out_channels=out_channels, features=features,
                                pool_size=pool_size, ablation_on_qk_channels=qk, precision=precision)
        if name == "UNet_FullResAttention":
            return UNet_FullResAttention(in_channels, out_channels, features, precision=precision)
        if name in ("TransformerUNet", "TransUNet"):   # reference :113-137
            print("正在創建官方版 TransUNet (R50-ViT-B_16)...")
            vit_config = get_r50_b16_config()
            img_size_config = config.get("dataset", {}).get("img_size", [224, 224])
            img_size = img_size_config[0] if isinstance(img_size_config, list) else img_size_config
            vit_config.n_classes = out_channels
            if in_channels != 3:
                print(f"注意：官方版 TransUNet 預設處理3通道輸入。您的 in_channels={in_channels}，模型會將單通道複製為3通道。")
            vit_config.patches.grid = (img_size // 16, img_size // 16)
            return TransUNet(config=vit_config, img_size=img_size, num_classes=out_channels, precision=precision)
        if name in _ZOO:
            cls, takes_pool = _ZOO[name]
            if takes_pool:
                return cls(in_channels, out_channels, features, pool_size, precision=precision)
            return cls(in_channels, out_channels, features, precision=precision)
        if name in _REFERENCE_ONLY:
            raise NotImplementedError(
                f"model {name!r} exists in the reference but is not built on the MI355X path yet "
                f"(built: {', '.join(_BUILT)})")
        raise ValueError(f"不支援的模型類型: {name}")

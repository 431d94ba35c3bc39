"""Utilities package (drop-in for the reference's utils/): metrics and the Trainer."""
from utils.metrics import BCEDiceLoss, calculate_metrics, dice_loss
from utils.trainer import Trainer

__all__ = ["BCEDiceLoss", "calculate_metrics", "dice_loss", "Trainer"]

"""Attention modules (reference flash_attn/modules/)."""

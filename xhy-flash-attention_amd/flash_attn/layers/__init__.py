"""Layers used by the attention modules (reference flash_attn/layers/)."""

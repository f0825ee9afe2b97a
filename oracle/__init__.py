"""ORACLE -- test infrastructure only (CPU restatements used as the checker; see attention_ref.py)."""

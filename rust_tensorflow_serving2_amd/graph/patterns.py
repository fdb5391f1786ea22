"""Subgraph pattern matchers for encoder (BERT-style) graphs.

Filled in with the BERT exporter; ResNet needs none of these.
"""
from __future__ import annotations


def match_gelu_subgraph(g, c, src):
    return None


def bert_passes():
    return []

"""Encoder-side pieces of the MI355X build (mirror of scenedino/models/backbones/)."""

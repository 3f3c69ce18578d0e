"""Test-only CPU oracle of the reference hot path (see xerus_ref.py header). Never imported by the product."""

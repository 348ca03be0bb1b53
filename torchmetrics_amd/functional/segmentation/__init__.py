"""Segmentation (reference ``F/segmentation/__init__.py`` exports nothing; utilities live in ``.utils``)."""

"""shai_amd.serving"""

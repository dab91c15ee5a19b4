"""shai_amd.utils"""

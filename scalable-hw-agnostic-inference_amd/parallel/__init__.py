"""shai_amd.parallel"""

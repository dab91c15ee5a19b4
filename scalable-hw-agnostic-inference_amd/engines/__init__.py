"""shai_amd.engines"""

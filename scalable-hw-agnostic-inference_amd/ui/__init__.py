"""shai_amd.ui"""

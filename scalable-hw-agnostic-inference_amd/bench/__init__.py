"""shai_amd.bench"""

"""shai_amd.models"""

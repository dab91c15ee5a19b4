"""shai_amd.autoscaler"""

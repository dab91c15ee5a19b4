"""shai_amd.router"""

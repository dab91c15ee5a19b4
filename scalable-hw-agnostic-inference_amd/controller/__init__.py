"""shai_amd.controller"""
